#!/bin/bash
# Half-precision inputs: SR apply slots per lane 2 vs 4 (SMQ_HALF_TV), 256M, interleaved.
# The SMQ_* environment knobs are read only by an experiment build (smq_common.h knob_env):
#   python tools/build_variant.py knobs -DSMQ_KNOBS=1   (this script then loads it via SMQ_LIB)
export SMQ_LIB="${SMQ_LIB:-${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}/exp/knobs/libsmq.so}"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do for dt in f16 bf16; do for m in 2 4; do
  SMQ_HALF_TV=$m SMQ_BENCH_DTYPE=$dt timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/htv_${dt}_${m}_$r.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/htv_${dt}_${m}_$r.log').read().strip().splitlines()[-1]);print('$dt tv=$m run $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done; done; done
