"""Per-size-class summary of the SmaQ launches of a `bench.py --config autograd_resnet34` profile
(tools/profile_round.sh: kernel trace + FETCH_SIZE / WRITE_SIZE passes).

Each codec call of the step is one smaq_fused_kernel<RM, V, TIN> launch of G workgroups (tensors
up to 8,388,611 elements) or statistics + apply launches above that. A class is (kernel, V, G);
for it: launches per training step, average / median duration, HBM bytes per launch from the PMC
passes ((2 * FETCH_SIZE + WRITE_SIZE) KiB, the gfx950 FETCH x2 correction) against the 8 B/elem
the single launch must move (x read once, y written once), and the class's share of the step.

python tools/autograd_profile.py <prof_dir> <out.json> [calls_per_step elements_per_step config]

With the last three arguments (the bench line's codec_calls_per_step, compressed_elements_per_step
and config) it also writes profiles/traffic_<config>.json, which bench.py reports as
roofline.traffic of that workload.
"""

import collections
import csv
import json
import re
import statistics
import sys

SMAQ = re.compile(r"smq::(smaq_\w+_kernel)(?:<([^>]*)>)?")
# SmartFP's launches (the single launch, or statistics + apply); the packed codec's kernels of a
# bench variant with packed saved activations are not counted
KERNELS = ("smaq_fused_kernel", "smaq_stats_kernel", "smaq_apply_kernel")


def classify(name, grid_threads, wg):
    m = SMAQ.search(name)
    if not m:
        return None
    kern, targs = m.group(1), m.group(2) or ""
    if kern not in KERNELS:
        return None
    g = int(grid_threads) // max(1, int(wg))
    if kern == "smaq_fused_kernel":
        v = int(targs.split(",")[1])
        return (kern, v, g)
    return (kern, 0, g)


def main():
    prof, out = sys.argv[1], sys.argv[2]
    calls_per_step = int(sys.argv[3]) if len(sys.argv) > 3 else 264
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{prof}/trace/run_kernel_trace.csv")):
        c = classify(r["Kernel_Name"], r["Grid_Size_X"], r["Workgroup_Size_X"])
        if c:
            dur[c].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    pmc = {}
    for cn, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f"{prof}/{sub}/run_counter_collection.csv")):
            if r["Counter_Name"] != cn:
                continue
            c = classify(r["Kernel_Name"], r["Grid_Size"], r["Workgroup_Size"])
            if c:
                acc[c].append(float(r["Counter_Value"]))
        pmc[cn] = {k: statistics.fmean(v) for k, v in acc.items()}
    fused_calls = sum(len(v) for k, v in dur.items() if k[0] == "smaq_fused_kernel")
    other = sum(len(v) for k, v in dur.items() if k[0] == "smaq_stats_kernel")
    steps = (fused_calls + other) / calls_per_step
    classes, tot_us = [], 0.0
    for k in sorted(dur, key=lambda k: (-k[1], -k[2], k[0])):
        d = dur[k]
        fetch, write = pmc["FETCH_SIZE"].get(k), pmc["WRITE_SIZE"].get(k)
        hbm = (2 * fetch + write) * 1024 if fetch is not None and write is not None else None
        # elements: the output is written once as fp32
        n = round(write * 1024 / 4) if write else None
        per_step = len(d) / steps
        avg = statistics.fmean(d)
        tot_us += per_step * avg
        row = {"kernel": k[0], "V": k[1], "workgroups": k[2], "launches": len(d),
               "launches_per_step": round(per_step, 2), "avg_us": round(avg, 3),
               "median_us": round(statistics.median(d), 3), "min_us": round(min(d), 3),
               "elements_est": n, "hbm_bytes_per_launch": None if hbm is None else round(hbm),
               "step_us": round(per_step * avg, 1)}
        if n and k[0] == "smaq_fused_kernel":
            row["alg_bytes_8B"] = 8 * n
            row["traffic_over_alg"] = round(hbm / (8 * n), 3) if hbm else None
            row["alg_tbps"] = round(8 * n / (avg * 1e-6) / 1e12, 3)
        classes.append(row)
    alg = sum(r.get("alg_bytes_8B", 0) * r["launches_per_step"] for r in classes)
    hbm = sum((r["hbm_bytes_per_launch"] or 0) * r["launches_per_step"] for r in classes)
    res = {"source": prof, "calls_per_step": calls_per_step, "steps_traced": round(steps, 2),
           "smaq_device_us_per_step": round(tot_us, 1),
           "alg_bytes_per_step_8B": round(alg), "hbm_bytes_per_step": round(hbm),
           "alg_tbps_over_device_time": round(alg / (tot_us * 1e-6) / 1e12, 3) if tot_us else None,
           "classes": classes}
    json.dump(res, open(out, "w"), indent=1)
    if len(sys.argv) > 5:
        import os

        config = sys.argv[5]
        tp = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                          f"traffic_{config}.json")
        json.dump({"source": out, "config": config, "calls_per_step": calls_per_step,
                   "elements_per_step": int(sys.argv[4]), "hbm_bytes_per_step": round(hbm),
                   "alg_bytes_per_step_8B": round(alg)}, open(tp, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "classes"}))
    for r in classes:
        print(r)


if __name__ == "__main__":
    main()
