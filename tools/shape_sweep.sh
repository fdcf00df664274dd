#!/bin/bash
# Headline: apply tiles in reverse (default) vs forward address order (SMQ_APPLY_REVERSE=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {  # label env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/sh_$l.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/sh_$l.log').read().strip().splitlines()[-1]);print('$l', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
}
for r in 1 2 3; do
  run rev_$r SMQ_APPLY_REVERSE=1
  run fwd_$r SMQ_APPLY_REVERSE=0
done
