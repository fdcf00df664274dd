#!/bin/bash
# Round-3 evidence, part 2: trace + FETCH / WRITE passes for the other configs and their bench lines.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
: > gpurun_out/r3b_bench_configs.jsonl
for c in fp8 s2fp8 multi packed smaq_sampled; do
  timeout -k 10 300 python3 bench.py --config $c >> gpurun_out/r3b_bench_configs.jsonl 2>> gpurun_out/r3b_bench.err || exit $?
done
for c in fp8 s2fp8 multi packed smaq_sampled; do
  bash tools/profile_round.sh r3b_$c $c 20 3 || exit $?
done
