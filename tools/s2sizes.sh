#!/bin/bash
# s2bench (single launch vs SMQ_S2FP8_SPLIT) over tensor sizes: 64K .. 4M elements.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for n in 65536 524288 1048576 3145728 4194304; do
  echo "n=$n $(S2B_N=$n timeout -k 10 120 python tools/s2bench.py 2>/dev/null | grep full)" || exit 1
done
