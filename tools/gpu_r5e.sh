#!/bin/bash
# Packed codec after the parallel re-code / big-block decode: its tests, the 256M bench line, the
# ResNet-34 packed-saved step and its kernel trace.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5e}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_packed.py tests/test_gpu_saved.py tests/test_gpu_optim.py > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_bench.jsonl
for c in packed autograd_resnet34; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
done
timeout -k 10 300 python -u tools/saved_profile.py > gpurun_out/${T}_saved_profile.txt 2>&1 || exit 1
head -2 gpurun_out/${T}_saved_profile.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${T}_saved -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/saved_profile.py > $GRAFT_REPO_ROOT/gpurun_out/${T}_saved_prof.log 2>&1 || exit 1
echo done
