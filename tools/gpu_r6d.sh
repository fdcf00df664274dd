#!/bin/bash
# Bisect: the autograd packed-codec identity test, then the packed / roundtrip-compress suites.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r6d}
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread "tests/test_gpu_optim.py::test_register_autograd_module_every_call_bitexact" > gpurun_out/${T}_a.log 2>&1; tail -n 3 gpurun_out/${T}_a.log
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_packed.py tests/test_gpu_roundtrip_compress.py > gpurun_out/${T}_b.log 2>&1; tail -n 8 gpurun_out/${T}_b.log
echo done
