"""Summarise a tools/profile_round.sh run into profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as produced)
  profiles/<tag>_summary.json       per-kernel avg duration (trace) and HBM bytes per launch (PMC)
  profiles/traffic_<config>.json    what bench.py reports as roofline.traffic

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE / WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE counts exactly half the bytes of a wide (16 B/lane) coalesced streaming read
(MI355X_MICROARCH.md §HBM), WRITE_SIZE is exact for 16 B/lane streaming stores.

python tools/pmc_traffic.py <prof_dir> <tag> [config]
"""

import collections
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SHORT = {
    "smaq_apply_kernel": "smaq_apply_kernel",
    "smaq_stats_kernel": "smaq_stats_kernel",
    "smaq_multi_stats_kernel": "smaq_multi_stats_kernel",
    "smaq_multi_apply_kernel": "smaq_multi_apply_kernel",
    "float_quant_kernel": "float_quant_kernel",
    "s2fp8_partial_kernel": "s2fp8_partial_kernel",
    "s2fp8_fused_kernel": "s2fp8_fused_kernel",
    "s2fp8_apply_kernel": "s2fp8_apply_kernel",
    "smaq_pack_kernel": "smaq_pack_kernel",
    "smaq_unpack_kernel": "smaq_unpack_kernel",
    "smaq_unpack_big_kernel": "smaq_unpack_big_kernel",
    "smaq_pack_block_kernel": "smaq_pack_block_kernel",
    "smaq_pack_var_kernel": "smaq_pack_var_kernel",
    "smaq_pack_scan_kernel": "smaq_pack_scan_kernel",
    "smaq_draw_stats_kernel": "smaq_draw_stats_kernel",
    "smaq_multi_draw_kernel": "smaq_multi_draw_kernel",
    "smaq_multi_final_kernel": "smaq_multi_final_kernel",
    "smaq_fused_kernel": "smaq_fused_kernel",
    "smaq_stats_small_kernel": "smaq_stats_small_kernel",
    "smq_fill_kernel": "smq_fill_kernel",
    "smaq_pack_recode_kernel": "smaq_pack_recode_kernel",
}


def short(name):
    for k, v in SHORT.items():
        if k in name:
            return v
    return None


def pmc(path, counter):
    out = collections.defaultdict(list)
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        s = short(r["Kernel_Name"])
        if s and r["Counter_Name"] == counter:
            out[s].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}


def main():
    prof, tag = sys.argv[1], sys.argv[2]
    config = sys.argv[3] if len(sys.argv) > 3 else "smaq"
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    stats_csv = os.path.join(prof, "trace", "run_kernel_stats.csv")
    shutil.copy(stats_csv, os.path.join(REPO, "profiles", f"{tag}_kernel_stats.csv"))
    dur = {}
    for r in csv.DictReader(open(stats_csv)):
        s = short(r["Name"])
        if s:
            dur[s] = dict(calls=int(r["Calls"]), avg_ms=float(r["AverageNs"]) / 1e6,
                          min_ms=float(r["MinNs"]) / 1e6, max_ms=float(r["MaxNs"]) / 1e6)
    fetch = pmc(os.path.join(prof, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = pmc(os.path.join(prof, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(dur) | set(fetch) | set(write)):
        rec = dict(dur.get(k, {}))
        if k in fetch:
            rec["fetch_size_kib"] = fetch[k]
            rec["read_bytes_per_launch"] = 2 * fetch[k] * 1024
        if k in write:
            rec["write_size_kib"] = write[k]
            rec["write_bytes_per_launch"] = write[k] * 1024
        if k in fetch and k in write:
            rec["hbm_bytes_per_launch"] = rec["read_bytes_per_launch"] + rec["write_bytes_per_launch"]
            if "avg_ms" in rec:
                rec["hbm_GBps"] = rec["hbm_bytes_per_launch"] / (rec["avg_ms"] * 1e-3) / 1e9
        kernels[k] = rec
    summary = dict(tag=tag, config=config, kernels=kernels,
                   note="HBM bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB per launch (gfx950 FETCH x2)")
    with open(os.path.join(REPO, "profiles", f"{tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    main_k = {"smaq": "smaq_apply_kernel", "smaq_sampled": "smaq_apply_kernel",
              "smaq_f16": "smaq_apply_kernel", "smaq_bf16": "smaq_apply_kernel",
              "fp8": "float_quant_kernel", "s2fp8": "s2fp8_fused_kernel",
              "multi": "smaq_multi_apply_kernel", "packed": "smaq_unpack_kernel"}[config]
    if main_k in kernels and "hbm_bytes_per_launch" in kernels[main_k]:
        # the workload the counters describe: bench.py reports them only for the same one
        elements = int(os.environ.get("SMQ_PROFILE_ELEMENTS", "0")) or {
            "fp8": 25690112, "s2fp8": 3145728, "multi": 42547220}.get(config, 1 << 28)
        dtype = {"smaq_f16": "f16", "smaq_bf16": "bf16"}.get(config, "f32")
        with open(os.path.join(REPO, "profiles", f"traffic_{config}.json"), "w") as f:
            json.dump(dict(source=f"profiles/{tag}_summary.json",
                           config=config.replace("_f16", "").replace("_bf16", ""),
                           elements=elements, dtype=dtype, kernel=main_k,
                           apply_bytes_per_launch=kernels[main_k]["hbm_bytes_per_launch"],
                           kernels={k: v.get("hbm_bytes_per_launch") for k, v in kernels.items()}),
                      f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
