#!/bin/bash
# float64 packed codec on the GPU (stream vs the restatement, round trip vs SmartFP), plus the
# fp64 unpacked tests (the statistics launch was factored out) and the packed suite.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5o}
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_packed_f64.py tests/test_f64.py tests/test_gpu_packed.py tests/test_cpu_packed.py > gpurun_out/${T}_tests.log 2>&1 || { tail -n 60 gpurun_out/${T}_tests.log; exit 1; }
tail -n 2 gpurun_out/${T}_tests.log
timeout -k 10 120 ./tools/launch_cost > gpurun_out/${T}_launch_cost.txt 2>&1 || exit 1
cat gpurun_out/${T}_launch_cost.txt
echo done
