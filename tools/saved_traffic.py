"""HBM traffic and device time of the packed-saved step's codec launches (measurement script, not
product), from `tools/profile_round.sh <tag> autograd_resnet34 T P --variants
smaq_eager_packed_saved` (kernel trace + separate FETCH_SIZE / WRITE_SIZE passes).

Classes: the forward calls' single launch that also packs (smaq_fused_kernel<..., PACK = true>,
by V), the grad-maps' plain single launch (PACK = false), the look-back packer of the calls above
4 groups per lane (smaq_pack_lb_kernel), the one-launch decode of the saved streams
(smaq_unpack_small_kernel). Per class: launches per step, average duration, HBM bytes per launch =
(2 * FETCH_SIZE + WRITE_SIZE) KiB (gfx950 FETCH x2 correction, MI355X_MICROARCH.md) and those bytes
over the duration.

The bench run also holds one counting step of plain SmartFP calls (264 launches) before the
variant's own steps: it is subtracted from the PACK = false class.

python tools/saved_traffic.py <prof_dir> <out.json> <trace_steps> <pmc_steps> [config]
(steps of the variant: 1 first + 1 memory + warm-up + timed, e.g. 15 for T=10 / W=3, 6 for P=3 /
W=1). With [config], also writes profiles/traffic_<config>_packed.json (what bench.py reports as
the packed-saved variant's traffic).
"""

import collections
import csv
import json
import os
import re
import statistics
import sys

NAME = re.compile(r"smq::(?:\(anonymous namespace\)::)?(\w+_kernel)(?:<([^>]*)>)?")
COUNTING_CALLS = 264


def classify(name):
    m = NAME.search(name)
    if not m:
        return None
    kern, targs = m.group(1), [a.strip() for a in (m.group(2) or "").split(",")]
    if kern == "smaq_fused_kernel":
        pack = len(targs) > 3 and targs[3] == "true"
        return (kern + ("[PACK]" if pack else ""), int(targs[1]))
    if kern in ("smaq_pack_lb_kernel", "smaq_unpack_small_kernel", "smaq_unpack_kernel",
                "smaq_pack_block_kernel", "smaq_pack_var_kernel", "smaq_stats_kernel",
                "smaq_apply_kernel"):
        return (kern, 0)
    return None


def main():
    prof, out = sys.argv[1], sys.argv[2]
    tsteps, psteps = float(sys.argv[3]), float(sys.argv[4])
    config = sys.argv[5] if len(sys.argv) > 5 else None
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{prof}/trace/run_kernel_trace.csv")):
        c = classify(r["Kernel_Name"])
        if c:
            dur[c].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    cnt = {}
    for cn, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        acc = collections.defaultdict(float)
        n = collections.Counter()
        for r in csv.DictReader(open(f"{prof}/{sub}/run_counter_collection.csv")):
            if r["Counter_Name"] != cn:
                continue
            c = classify(r["Kernel_Name"])
            if c:
                acc[c] += float(r["Counter_Value"])
                n[c] += 1
        cnt[cn] = (acc, n)
    rows, tot_us, tot_b = [], 0.0, 0.0
    for k in sorted(dur, key=lambda k: (k[0], k[1])):
        d = dur[k]
        fa, fn = cnt["FETCH_SIZE"]
        wa, wn = cnt["WRITE_SIZE"]
        hbm = None
        if fn[k] and wn[k]:
            hbm = (2 * fa[k] / fn[k] + wa[k] / wn[k]) * 1024
        avg = statistics.fmean(d)
        rows.append({"kernel": k[0], "V": k[1], "launches_traced": len(d), "avg_us": round(avg, 3),
                     "median_us": round(statistics.median(d), 3),
                     "hbm_bytes_per_launch": None if hbm is None else round(hbm),
                     "hbm_gbps": None if hbm is None else round(hbm / (avg * 1e-6) / 1e9, 1),
                     "fetch_kib_per_launch": round(fa[k] / fn[k], 1) if fn[k] else None,
                     "write_kib_per_launch": round(wa[k] / wn[k], 1) if wn[k] else None})
    # per step: the trace's launches over its steps; the plain launches of the counting step out
    plain_total = sum(r["launches_traced"] for r in rows if r["kernel"] == "smaq_fused_kernel")
    for r in rows:
        n = r["launches_traced"]
        if r["kernel"] == "smaq_fused_kernel" and plain_total:
            n -= COUNTING_CALLS * n / plain_total  # (the counting step's share of this class)
        r["launches_per_step"] = round(n / tsteps, 2)
        r["device_us_per_step"] = round(r["launches_per_step"] * r["avg_us"], 1)
        tot_us += r["device_us_per_step"]
        if r["hbm_bytes_per_launch"] is not None:
            tot_b += r["launches_per_step"] * r["hbm_bytes_per_launch"]
    res = {"source": prof, "variant": "smaq_eager_packed_saved", "trace_steps": tsteps,
           "pmc_steps": psteps, "codec_device_us_per_step": round(tot_us, 1),
           "codec_hbm_bytes_per_step": round(tot_b),
           "codec_hbm_gbps_over_device_time": round(tot_b / (tot_us * 1e-6) / 1e9, 1) if tot_us else None,
           "classes": rows}
    json.dump(res, open(out, "w"), indent=1)
    if config:
        tp = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                          f"traffic_{config}_packed.json")
        json.dump({"source": out, "config": config, "variant": "smaq_eager_packed_saved",
                   "hbm_bytes_per_step": round(tot_b), "device_us_per_step": round(tot_us, 1)},
                  open(tp, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "classes"}))
    for r in rows:
        print(r)


if __name__ == "__main__":
    main()
