#!/bin/bash
# Interleaved per-call times of the single-launch SmaQ (tools/defer_sweep.py at 1M / 4M / 8M) for
# library builds exp/<name>/libsmq.so (tools/build_variant.py), 3 rounds.
# Usage: bash tools/fstore_ab.sh <name>...
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
for r in 1 2 3; do
  for v in "$@"; do
    out=$(SMQ_LIB="$R/exp/$v/libsmq.so" DS_SIZES=${FA_SIZES:-1048576,4194304,8388608} timeout -k 10 120 python3 tools/defer_sweep.py 2>/dev/null) || exit 1
    echo "round $r $v: $(echo "$out" | tr '\n' ' ')"
  done
done
