#!/bin/bash
# Packer: var kernel with early scratch loads; constants pinned in VGPRs in the code kernel.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5q}
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_packed.py tests/test_gpu_saved.py tests/test_packed_f64.py > gpurun_out/${T}_tests.log 2>&1 || { tail -n 60 gpurun_out/${T}_tests.log; exit 1; }
tail -n 2 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_bench.jsonl
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --config packed --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/${T}_bench.jsonl'):
    d=json.loads(l); print(d['config'].get('workload'), d['ms_per_step'], d.get('compress_ms'), d.get('decompress_ms'))
"
bash tools/profile_round.sh ${T}_packed packed > /dev/null || exit 1
echo done
