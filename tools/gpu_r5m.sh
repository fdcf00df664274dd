#!/bin/bash
# Packer without the fill and scan launches (group sums cleared by the statistics launch, group
# prefixes summed by the var kernel), one-op relu: parity, bench, profiles.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5m}
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_smaq.py tests/test_gpu_packed.py tests/test_gpu_saved.py tests/test_gpu_graph_safe.py tests/test_gpu_fused.py tests/test_gpu_multi.py > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_bench.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config packed --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
  SMQ_BENCH_DTYPE=f16 timeout -k 10 300 python -u bench.py --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
done
timeout -k 10 300 python -u bench.py --config autograd_resnet34 --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/${T}_bench.jsonl'):
    d=json.loads(l); print(d['config'].get('workload'), d['dtype'], d['ms_per_step'], d.get('compress_ms'), d['roofline']['achieved'], {k: v for k, v in d.items() if k.startswith('variant') or k == 'variants'})
"
bash tools/profile_round.sh ${T}_packed packed > /dev/null || exit 1
echo done
