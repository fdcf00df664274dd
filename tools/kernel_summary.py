"""Per-kernel device time of a rocprofv3 --kernel-trace run (measurement script, not product):
calls per step, p50 / p90 / max duration, ms per step, for the library's kernels by name and
everything else as "other".

python tools/kernel_summary.py <prof_dir> <out.json> <steps> [note]

<prof_dir> holds run_kernel_trace.csv (rocprofv3 -d <prof_dir> -o run --output-format csv).
<steps>: the steps the traced program ran in total, warm-up included (tools/saved_trace.py N runs
N + 3): every launch's count and time are divided by it.
"""

import collections
import csv
import glob
import json
import os
import re
import statistics
import sys

NAME = re.compile(r"smq::(?:\(anonymous namespace\)::)?(\w+_kernel)")


def main():
    prof, out, steps = sys.argv[1], sys.argv[2], float(sys.argv[3])
    note = sys.argv[4] if len(sys.argv) > 4 else ""
    paths = glob.glob(os.path.join(prof, "**", "*kernel_trace.csv"), recursive=True)
    if not paths:
        sys.exit(f"no kernel_trace.csv under {prof}")
    dur = collections.defaultdict(list)
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                m = NAME.search(r["Kernel_Name"])
                key = m.group(1) if m else "other"
                dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    res = {}
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        res[k] = {"calls_per_step": round(len(v) / steps, 2),
                  "p50_us": round(statistics.median(v), 3),
                  "p90_us": round(v[int(0.9 * (len(v) - 1))], 3),
                  "max_us": round(v[-1], 3),
                  "ms_per_step": round(sum(v) / steps / 1e3, 4)}
    codec = sum(d["ms_per_step"] for k, d in res.items() if k != "other")
    with open(out, "w") as f:
        json.dump({"note": note, "steps": steps, "codec_ms_per_step": round(codec, 4),
                   "kernels": res}, f, indent=1)
    print(json.dumps({"codec_ms_per_step": round(codec, 4),
                      **{k: (d["calls_per_step"], d["p50_us"], d["ms_per_step"])
                         for k, d in res.items()}}))


if __name__ == "__main__":
    main()
