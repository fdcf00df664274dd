#!/bin/bash
# Single launch (DS_FLAGS=0) against the deferred two-launch path (DS_FLAGS=1), interleaved rounds,
# per tensor size (tools/defer_sweep.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export DS_SIZES=${DS_SIZES:-65536,262144,1048576,2097152,4194304,6291456,8388608}
for r in 1 2; do
  for f in 1 0; do
    DS_FLAGS=$f timeout -k 10 120 python tools/defer_sweep.py || exit 1
  done
done
