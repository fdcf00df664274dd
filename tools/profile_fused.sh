#!/bin/bash
# rocprofv3 evidence for the single-launch SmaQ (smaq_fused_kernel): a kernel trace + stats of
# back-to-back calls at one size per run (tools/defer_sweep.py), then FETCH_SIZE / WRITE_SIZE
# passes (each its own run, never combined with tracing). Outputs under gpurun_out/prof_<tag>_<n>.
# Usage: bash tools/profile_fused.sh <tag> [sizes...]
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r4b_fused}; shift
SIZES=${*:-1048576 4194304 8388608}
cd /tmp && export TMPDIR=/tmp
for n in $SIZES; do
  OUT="$REPO/gpurun_out/prof_${TAG}_$n"
  mkdir -p "$OUT"
  export DS_SIZES=$n DS_CALLS=100 DS_FLAGS=0
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$REPO/tools/defer_sweep.py" > "$OUT/trace.log" 2>&1 || exit $?
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d "$OUT/${c,,}" -o run --output-format csv -- \
      python3 "$REPO/tools/defer_sweep.py" > "$OUT/$c.log" 2>&1 || exit $?
  done
  tail -n 1 "$OUT/trace.log"
done
