#!/bin/bash
# The GPU test suite (or the given test files / -k selection) on a gpurun box, one process, each
# test under a thread timeout; the log under gpurun_out/<tag>_gpu_tests.log, the failing tail on
# stdout. Then smoke() unless SMQ_NO_SMOKE=1.
# Usage: bash tools/gpu_suite.sh <tag> [pytest args...]   (default args: tests)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG=$1; shift
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(tests)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread "${ARGS[@]}" -m gpu \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -n 40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -n 2 gpurun_out/${TAG}_gpu_tests.log
[ "${SMQ_NO_SMOKE:-0}" = 1 ] && exit 0
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -n 1
