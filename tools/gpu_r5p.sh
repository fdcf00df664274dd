#!/bin/bash
# Multi-tensor SmaQ with the per-tensor finalisation inside the apply launch: the multi suite
# (148 C5 tensors against per-tensor calls), bench lines, profile.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5p}
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_multi.py > gpurun_out/${T}_tests.log 2>&1 || { tail -n 60 gpurun_out/${T}_tests.log; exit 1; }
tail -n 2 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_bench.jsonl
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --config multi --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/${T}_bench.jsonl'):
    d=json.loads(l); print(d['config'].get('workload'), d['ms_per_step'], d['roofline']['achieved'])
"
bash tools/profile_round.sh ${T}_multi multi > /dev/null || exit 1
echo done
