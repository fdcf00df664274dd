#!/bin/bash
# The GPU suite and smoke at the round's last commit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r6q_gpu_tests.log 2>&1 || { tail -n 30 gpurun_out/r6q_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/r6q_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -n 1
