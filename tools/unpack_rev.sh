#!/bin/bash
# Packed decoder block order: forward (0) vs reverse (1), kernel trace each, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for m in 0 1 0 1; do
  SMQ_UNPACK_REVERSE=$m bash tools/ktrace.sh ur$m packed 20 | grep -E "unpack|emit" | cut -c1-170 || exit 1
  tail -1 gpurun_out/kt_ur$m/bench.log | cut -c1-200
done
