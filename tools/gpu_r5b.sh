#!/bin/bash
# Round 5: the whole GPU suite, the host-path cost, and the bench lines the host path moves.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5b}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 2 gpurun_out/${T}_tests.log
timeout -k 10 200 python -u tools/host_cost_smaq.py > gpurun_out/${T}_hc_smaq.txt 2>&1 || { tail -20 gpurun_out/${T}_hc_smaq.txt; exit 1; }
head -3 gpurun_out/${T}_hc_smaq.txt
: > gpurun_out/${T}_bench.jsonl
for c in autograd_resnet34 autograd s2fp8; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
done
echo done
