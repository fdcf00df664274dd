#!/bin/bash
# One PMC pass (no tracing domains) over a bench config; prints per-kernel averages of the counters.
# Usage: bash tools/prof_pmc.sh <name> "<counters>" <bench args...>
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
NAME=$1; CTRS=$2; shift 2
OUT="$REPO/gpurun_out/pmc_$NAME"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d "$OUT" -o run --output-format csv -- python3 "$REPO/bench.py" --no-cpu-baseline "$@" > "$OUT/bench.log" 2>&1
rc=$?
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    acc[(r["Kernel_Name"][:70], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:70s} {c:24s} {sum(v)/len(v):16.1f}")
PY
exit $rc
