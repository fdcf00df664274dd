#!/bin/bash
# Headline bench: event markers inside the timed steps (old) vs in a separate roofline pass (new).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {  # label env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/sh_$l.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/sh_$l.log').read().strip().splitlines()[-1]);print('$l', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
}
for r in 1 2 3; do
  run sep_$r SMQ_BENCH_EVENTS_IN_TIMED=0
  run in_$r SMQ_BENCH_EVENTS_IN_TIMED=1
done
