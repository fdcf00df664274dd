#!/bin/bash
# Packed round trip: statistics with nt loads (default at 1 GiB) vs plain (SMQ_STATS_NT_MIN_MB).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {  # label env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config packed --steps 20 --warmup 3 > gpurun_out/sh_$l.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/sh_$l.log').read().strip().splitlines()[-1]);print('$l', d['value'], d['ms_per_step'], d['compress_ms'], d['decompress_ms'])"
}
for r in 1 2 3; do
  run nt_$r SMQ_STATS_NT_MIN_MB=512
  run plain_$r SMQ_STATS_NT_MIN_MB=100000
done
