#!/bin/bash
# Headline bench three times (20 steps each) plus the deferred-size sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/h3_$r.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/h3_$r.log').read().strip().splitlines()[-1]);print('run $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
DS_SIZES=1048576,4194304,16777216 timeout -k 10 120 python tools/defer_sweep.py || exit 1
