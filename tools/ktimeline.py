"""Per-kernel durations and the idle gap before each kernel, from a rocprofv3 kernel trace CSV
(measurement aid). Usage: python tools/ktimeline.py <dir with *kernel_trace.csv> [name filter]"""

import collections
import csv
import glob
import os
import sys

import numpy as np


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    prev_end = None
    for r in rows:
        name = r["Kernel_Name"].split("(")[0][:70]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if flt in name:
            dur[name].append(e - s)
            if prev_end is not None:
                gap[name].append(s - prev_end)
        prev_end = e
    for k in dur:
        d = np.array(dur[k]) / 1e3
        g = np.array(gap[k]) / 1e3 if gap[k] else np.array([0.0])
        print(f"{k:70s} n={d.size:6d} dur med {np.median(d):8.2f} us  p10 {np.percentile(d, 10):8.2f}"
              f"  gap-before med {np.median(g):7.2f} us p10 {np.percentile(g, 10):7.2f}")


if __name__ == "__main__":
    main()
