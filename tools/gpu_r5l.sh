#!/bin/bash
# Quad-run draws (scalar quad base) in the apply and the packer: parity, bench, profiles.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5l}
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_smaq.py tests/test_gpu_packed.py tests/test_gpu_saved.py tests/test_gpu_graph_safe.py > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
timeout -k 10 120 ./tools/launch_cost > gpurun_out/${T}_launch_cost.txt 2>&1 || exit 1
cat gpurun_out/${T}_launch_cost.txt
: > gpurun_out/${T}_bench.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config packed --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
  SMQ_BENCH_DTYPE=f16 timeout -k 10 300 python -u bench.py --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/${T}_bench.jsonl'):
    d=json.loads(l); print(d['config'].get('workload'), d['dtype'], d['ms_per_step'], d['roofline']['achieved'])
"
bash tools/profile_round.sh ${T}_packed packed > /dev/null || exit 1
echo done
