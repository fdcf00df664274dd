#!/bin/bash
# Deferred statistics on/off (SMQ_DEFER_MAX_N=0), interleaved rounds, per tensor size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  echo "== round $r: off"; SMQ_DEFER_MAX_N=0 timeout -k 10 120 python tools/defer_sweep.py || exit 1
  echo "== round $r: on"; timeout -k 10 120 python tools/defer_sweep.py || exit 1
done
