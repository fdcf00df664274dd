#!/bin/bash
# Kernel trace + stats of one bench config (no PMC): prints the per-kernel summary.
# Usage: bash tools/prof_trace.sh <name> <bench args...>
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
NAME=$1; shift
OUT="$REPO/gpurun_out/tr_$NAME"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- python3 "$REPO/bench.py" --no-cpu-baseline "$@" > "$OUT/bench.log" 2>&1
rc=$?
tail -n 1 "$OUT/bench.log" | cut -c1-400
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    print(f"{r['Name'][:90]:90s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:9.2f}")
PY
exit $rc
