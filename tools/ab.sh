#!/bin/bash
# Interleaved A/B of the current build (lib/libsmq.so) against a baseline build
# (lib/ab/libsmq_base.so) on one bench config. Usage: bash tools/ab.sh <config> [rounds] [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/smart-quantization_amd/lib
C=$1; R=${2:-3}; shift 2
for r in $(seq 1 $R); do for v in base new; do
  lib=$L/libsmq.so; [ $v = base ] && lib=$L/ab/libsmq_base.so
  SMQ_LIB=$lib timeout -k 10 200 python bench.py --config $C --no-cpu-baseline "$@" > gpurun_out/ab_${C}_${v}_$r.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_${C}_${v}_$r.log').read().strip().splitlines()[-1]);print('$C $v run $r', d['value'], d['ms_per_step'])"
done; done
