#!/bin/bash
# A/B of the plain-load tail of the nt statistics sweep (SMQ_STATS_PLAIN_TAIL_MB), headline bench,
# interleaved rounds. Prints ms/step and the event-timed apply per setting.
# The SMQ_* environment knobs are read only by an experiment build (smq_common.h knob_env):
#   python tools/build_variant.py knobs -DSMQ_KNOBS=1   (this script then loads it via SMQ_LIB)
export SMQ_LIB="${SMQ_LIB:-${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}/exp/knobs/libsmq.so}"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for mb in ${TAILS:-0 128 192 256}; do
    out=$(SMQ_STATS_PLAIN_TAIL_MB=$mb timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline 2>/dev/null) || exit 1
    echo "tail=$mb $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["avg_launch_ms"])')"
  done
done
