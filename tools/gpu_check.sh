#!/bin/bash
# One config after a kernel change: the given GPU test files, two bench lines of the config, then
# its kernel trace + FETCH / WRITE passes (tools/profile_round.sh <tag> <config>).
# Usage: bash tools/gpu_check.sh <tag> <config> <test files...>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG=$1; CONFIG=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" -m gpu \
  > gpurun_out/t_$TAG.log 2>&1
rc=$?
tail -n 3 gpurun_out/t_$TAG.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/${TAG}_bench.jsonl
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --config $CONFIG --no-cpu-baseline >> gpurun_out/${TAG}_bench.jsonl \
    2> gpurun_out/${TAG}_bench.err || exit $?
done
cut -c1-250 gpurun_out/${TAG}_bench.jsonl
bash tools/profile_round.sh $TAG $CONFIG
