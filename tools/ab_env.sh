#!/bin/bash
# A/B of environment settings on one bench config, interleaved rounds.
# Usage: bash tools/ab_env.sh <rounds> "<bench args>" "<env A>" "<env B>" ...
# The SMQ_* environment knobs are read only by an experiment build (smq_common.h knob_env):
#   python tools/build_variant.py knobs -DSMQ_KNOBS=1   (this script then loads it via SMQ_LIB)
export SMQ_LIB="${SMQ_LIB:-${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}/exp/knobs/libsmq.so}"
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
ROUNDS=$1; ARGS=$2; shift 2
for r in $(seq 1 "$ROUNDS"); do
  for envs in "$@"; do
    line=$(env $envs timeout -k 10 180 python3 "$R/bench.py" --no-cpu-baseline $ARGS 2>/dev/null | tail -n 1) || exit 1
    ms=$(python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step'], d.get('roofline',{}).get('achieved'))" "$line")
    echo "round $r [$envs] $ms"
  done
done
