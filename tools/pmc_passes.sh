#!/bin/bash
# SQ/LDS PMC passes (no tracing domains combined) for one bench config; one rocprofv3 run per pass.
# Usage: bash tools/pmc_passes.sh <tag> <config> "<counters pass 1>" ["<counters pass 2>" ...]
# A counter-name error ends that pass only; a fault / abort / timeout ends the script.
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; CONFIG=$2; shift 2
OUT="$REPO/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "$@"; do
  i=$((i + 1))
  echo "== pass $i: $ctrs"
  timeout -k 10 600 rocprofv3 --pmc $ctrs -d "$OUT/p$i" -o run --output-format csv -- \
    python3 "$REPO/bench.py" --config "$CONFIG" --no-cpu-baseline --steps 3 --warmup 1 \
    > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"; tail -n 3 "$OUT/p$i.log" | cut -c1-300
  case $rc in 0|1|2) ;; *) echo "stopping (rc=$rc)"; exit $rc ;; esac
done
