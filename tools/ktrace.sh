#!/bin/bash
# rocprofv3 kernel trace + stats of one bench config; prints the per-kernel summary.
# Usage: bash tools/ktrace.sh <tag> <config> [steps] [extra bench args...]
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; CONFIG=$2; STEPS=${3:-100}; shift 3
OUT="$REPO/gpurun_out/kt_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- \
  python3 "$REPO/bench.py" --config "$CONFIG" --no-cpu-baseline --steps "$STEPS" --warmup 10 "$@" \
  > "$OUT/bench.log" 2>&1 || exit $?
tail -n 1 "$OUT/bench.log" | cut -c1-400
f=$(find "$OUT" -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if int(r["Calls"]) >= 10:
        print(f'{r["Name"][:90]:90s} calls={r["Calls"]:>6} avg_us={float(r["AverageNs"])/1e3:9.2f} min_us={float(r["MinNs"])/1e3:9.2f}')
PY
