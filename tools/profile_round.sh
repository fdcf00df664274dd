#!/bin/bash
# rocprofv3 evidence for the bench line: kernel trace + stats, then separate PMC passes for
# FETCH_SIZE and WRITE_SIZE (never combined with tracing domains). Outputs under gpurun_out/prof_*.
# Usage: bash tools/profile_round.sh <tag> [bench args...]
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r01}; shift
ARGS=${*:---steps 20 --warmup 3 --no-cpu-baseline}
OUT="$REPO/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 3 "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$REPO/bench.py" $ARGS
run fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 "$REPO/bench.py" --steps 5 --warmup 1 --no-cpu-baseline ${PMC_EXTRA}
run write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 "$REPO/bench.py" --steps 5 --warmup 1 --no-cpu-baseline ${PMC_EXTRA}
find "$OUT" -name "*.csv" | head -50
