#!/bin/bash
# A/B of two library builds (SMQ_LIB) on bench configs, interleaved rounds.
# Usage: bash tools/ab_lib.sh <libA> <libB> <rounds> "<config spec>"...
#   spec: "<label>|<env assignments>|<bench args>"
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
A=$1; B=$2; ROUNDS=$3; shift 3
mkdir -p "$R/gpurun_out"
for r in $(seq 1 "$ROUNDS"); do
  for spec in "$@"; do
    IFS='|' read -r label envs args <<< "$spec"
    for lib in "$A" "$B"; do
      line=$(env $envs SMQ_LIB="$lib" timeout -k 10 180 python3 "$R/bench.py" --no-cpu-baseline $args 2>/dev/null | tail -n 1) || exit 1
      ms=$(python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step'], d.get('roofline',{}).get('achieved'), d.get('roofline',{}).get('avg_launch_ms'))" "$line")
      echo "round $r $label $(basename $(dirname $lib)) $ms"
    done
  done
done
