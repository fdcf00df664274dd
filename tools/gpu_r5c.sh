#!/bin/bash
# Round 5: saved-activation / host-path tests, then the bench lines and profiles the quad-hash
# draws move (packed compress, half-input apply, headline, autograd).
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5c}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_saved.py tests/test_gpu_hostpath.py > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_bench.jsonl
timeout -k 10 300 python -u bench.py >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
for c in packed autograd_resnet34 multi; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
done
for d in f16 bf16; do
  SMQ_BENCH_DTYPE=$d timeout -k 10 300 python -u bench.py --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
done
bash tools/profile_round.sh ${T}_packed packed > /dev/null || exit 1
SMQ_BENCH_DTYPE=f16 bash tools/profile_round.sh ${T}_smaq_f16 smaq > /dev/null || exit 1
SMQ_BENCH_DTYPE=bf16 bash tools/profile_round.sh ${T}_smaq_bf16 smaq > /dev/null || exit 1
echo done
