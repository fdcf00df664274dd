#!/bin/bash
# The C backward decode of saved streams: saved-mode GPU tests and the saved-mode A/B.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r6p}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_saved.py tests/test_gpu_optim.py > gpurun_out/${T}_tests.log 2>&1 || { tail -n 30 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u tools/saved_ab.py 5 > gpurun_out/${T}_saved_ab.txt 2>&1 || { tail -n 20 gpurun_out/${T}_saved_ab.txt; exit 1; }
head -n 5 gpurun_out/${T}_saved_ab.txt | cut -c1-300
echo done
