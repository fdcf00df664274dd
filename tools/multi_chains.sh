#!/bin/bash
# C5 multi-tensor bench, three runs, plus its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --config multi --steps 100 --warmup 10 > gpurun_out/mc_$r.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/mc_$r.log').read().strip().splitlines()[-1]);print('run $r', d['value'], d['ms_per_step'])"
done
bash tools/ktrace.sh mc multi 50 | grep smq | cut -c1-170
