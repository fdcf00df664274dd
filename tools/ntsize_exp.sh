#!/bin/bash
# Statistics-load policy vs tensor size: SMQ_STATS_NT_MIN_MB=0 (always nt) vs 100000 (never).
# The SMQ_* environment knobs are read only by an experiment build (smq_common.h knob_env):
#   python tools/build_variant.py knobs -DSMQ_KNOBS=1   (this script then loads it via SMQ_LIB)
export SMQ_LIB="${SMQ_LIB:-${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}/exp/knobs/libsmq.so}"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for e in 16777216 67108864 268435456; do for r in 1 2; do for m in 0 100000; do
  SMQ_STATS_NT_MIN_MB=$m timeout -k 10 200 python bench.py --elements $e --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/nts_${e}_${m}_$r.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/nts_${e}_${m}_$r.log').read().strip().splitlines()[-1]);print('n=$e nt_min=$m run $r', d['value'], d['ms_per_step'])"
done; done; done
