#!/bin/bash
# tools/tail_exp.sh at the driver's bench length (20 steps, 3 warm-up).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2 3; do
  for mb in 0 256; do
    out=$(SMQ_STATS_PLAIN_TAIL_MB=$mb timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null) || exit 1
    echo "tail=$mb $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["avg_launch_ms"])')"
  done
done
