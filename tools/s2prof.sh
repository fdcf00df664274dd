#!/bin/bash
# S2FP8 (C4) kernel timeline under rocprofv3: durations and launch gaps, eager and graph replay.
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-s2}
OUT="$REPO/gpurun_out/kt_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- \
  python3 "$REPO/bench.py" --config s2fp8 --no-cpu-baseline --steps 480 --warmup 10 \
  > "$OUT/bench.log" 2>&1 || exit $?
python3 "$REPO/tools/ktimeline.py" "$OUT" s2fp8
