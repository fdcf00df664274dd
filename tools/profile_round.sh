#!/bin/bash
# rocprofv3 evidence for a bench config: kernel trace + stats, then separate PMC passes for
# FETCH_SIZE and WRITE_SIZE (never combined with tracing domains). Outputs under gpurun_out/prof_*.
# Usage: bash tools/profile_round.sh <tag> <config> [trace steps] [pmc steps] [extra bench args...]
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r01}
CONFIG=${2:-smaq}
TSTEPS=${3:-20}
PSTEPS=${4:-5}
shift $(( $# < 4 ? $# : 4 ))
EXTRA="$*"
OUT="$REPO/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="$REPO/bench.py --config $CONFIG --no-cpu-baseline $EXTRA"
run trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $B --steps $TSTEPS --warmup 3
run fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 $B --steps $PSTEPS --warmup 1
run write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 $B --steps $PSTEPS --warmup 1
