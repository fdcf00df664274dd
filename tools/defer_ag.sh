#!/bin/bash
# Autograd config (VGG b128, SmaQ on every activation and gradient) with deferred statistics
# off (SMQ_DEFER_MAX_N=0) and on, interleaved.
# The SMQ_* environment knobs are read only by an experiment build (smq_common.h knob_env):
#   python tools/build_variant.py knobs -DSMQ_KNOBS=1   (this script then loads it via SMQ_LIB)
export SMQ_LIB="${SMQ_LIB:-${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}/exp/knobs/libsmq.so}"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do for m in 0 default; do
  if [ $m = 0 ]; then export SMQ_DEFER_MAX_N=0; else unset SMQ_DEFER_MAX_N; fi
  timeout -k 10 240 python bench.py --config autograd > gpurun_out/dag_${m}_$r.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/dag_${m}_$r.log').read().strip().splitlines()[-1]);print('defer=$m run $r', d['value'], d['ms_per_step'], {k: v for k, v in d.items() if 'ms' in k})"
done; done
