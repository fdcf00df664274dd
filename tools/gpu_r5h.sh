#!/bin/bash
# Packed codec after folding the group-sum fill into the scan and the re-code into the var launch.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5h}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_packed.py tests/test_gpu_saved.py > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_bench.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config packed --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
done
bash tools/profile_round.sh ${T}_packed packed > /dev/null || exit 1
echo done
