#!/bin/bash
# A/B of two builds of libsmq (SMQ_LIB: libsmq.so vs libsmq_nt.so) on several bench configs,
# interleaved. Usage: bash tools/stores_exp.sh <config> [rounds] [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=smart-quantization_amd/lib
C=$1; R=${2:-2}; shift 2
for r in $(seq 1 $R); do for v in sc nt; do
  lib=$L/libsmq.so; [ $v = nt ] && lib=$L/libsmq_nt.so
  SMQ_LIB=$PWD/$lib timeout -k 10 200 python bench.py --config $C --no-cpu-baseline "$@" > gpurun_out/st_${C}_${v}_$r.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/st_${C}_${v}_$r.log').read().strip().splitlines()[-1]);print('$C $v run $r', d['value'], d['ms_per_step'])"
done; done
