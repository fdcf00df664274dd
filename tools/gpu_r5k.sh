#!/bin/bash
# Half-input apply with the two-op fp32 quotient (smq_half_quot_split): parity, A/B against the
# fp64 form (knobs build, SMQ_HALF_QF=0), profiles of the fp16 / bf16 headline, launch cost.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5k}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_smaq.py -k "half or golden" > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
timeout -k 10 120 ./tools/launch_cost > gpurun_out/${T}_launch_cost.txt 2>&1 || exit 1
cat gpurun_out/${T}_launch_cost.txt
bash tools/ab_env.sh 3 "--config smaq" "SMQ_BENCH_DTYPE=f16 SMQ_HALF_QF=0" "SMQ_BENCH_DTYPE=f16 SMQ_HALF_QF=1" "SMQ_BENCH_DTYPE=bf16 SMQ_HALF_QF=0" "SMQ_BENCH_DTYPE=bf16 SMQ_HALF_QF=1" > gpurun_out/${T}_ab.txt 2>&1 || exit 1
cat gpurun_out/${T}_ab.txt
SMQ_BENCH_DTYPE=f16 bash tools/profile_round.sh ${T}_f16 smaq > /dev/null || exit 1
SMQ_BENCH_DTYPE=bf16 bash tools/profile_round.sh ${T}_bf16 smaq > /dev/null || exit 1
echo done
