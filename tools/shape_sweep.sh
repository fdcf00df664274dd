#!/bin/bash
# Half-precision inputs: statistics grid-stride (default) vs tile-stride, interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {  # label env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/sh_$l.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/sh_$l.log').read().strip().splitlines()[-1]);print('$l', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
}
for r in 1 2 3; do for dt in bf16 f16; do
  run ${dt}_grid_$r SMQ_BENCH_DTYPE=$dt
  run ${dt}_tile_$r SMQ_BENCH_DTYPE=$dt SMQ_STATS_TILE_HALF=1
done; done
