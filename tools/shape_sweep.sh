#!/bin/bash
# bf16 / fp16 inputs on two builds (SMQ_LIB), interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/smart-quantization_amd/lib
run() {  # label env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/sh_$l.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/sh_$l.log').read().strip().splitlines()[-1]);print('$l', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
}
for r in 1 2; do
  run bf16_new_$r SMQ_BENCH_DTYPE=bf16 SMQ_LIB=$L/libsmq.so
  run bf16_old_$r SMQ_BENCH_DTYPE=bf16 SMQ_LIB=$L/libsmq_nt.so
done
