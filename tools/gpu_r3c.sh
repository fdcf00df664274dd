#!/bin/bash
# Round-3 closing evidence: the whole GPU suite, the default bench line (with its CPU baseline), every
# config's line, then kernel traces + FETCH / WRITE passes (tools/profile_round.sh) of the headline,
# its fp16 variant, the packed codec and S2FP8. Outputs under gpurun_out/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/t_r3c.log 2>&1
rc=$?
tail -n 3 gpurun_out/t_r3c.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.err || exit $?
cut -c1-300 gpurun_out/r3c_bench.json
: > gpurun_out/r3c_bench_configs.jsonl
for c in fp8 s2fp8 multi packed; do
  timeout -k 10 240 python -u bench.py --config $c --no-cpu-baseline >> gpurun_out/r3c_bench_configs.jsonl \
    2> gpurun_out/r3c_bench_$c.err || exit $?
done
for d in f16 bf16; do
  SMQ_BENCH_DTYPE=$d timeout -k 10 240 python -u bench.py --no-cpu-baseline \
    >> gpurun_out/r3c_bench_configs.jsonl 2> gpurun_out/r3c_bench_$d.err || exit $?
done
cut -c1-200 gpurun_out/r3c_bench_configs.jsonl
bash tools/profile_round.sh r3c_smaq smaq || exit $?
SMQ_BENCH_DTYPE=f16 bash tools/profile_round.sh r3c_smaq_f16 smaq || exit $?
bash tools/profile_round.sh r3c_packed packed || exit $?
bash tools/profile_round.sh r3c_s2fp8 s2fp8 || exit $?
