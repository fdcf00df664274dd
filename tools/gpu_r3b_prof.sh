#!/bin/bash
# Round-3 evidence, part 1: the default bench line, then trace + FETCH / WRITE passes for the
# headline and the half-input variants.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/r3b_bench.json 2> gpurun_out/r3b_bench.err || exit $?
tail -n 1 gpurun_out/r3b_bench.json | cut -c1-300
bash tools/profile_round.sh r3b_smaq smaq 20 3 || exit $?
SMQ_BENCH_DTYPE=f16 bash tools/profile_round.sh r3b_smaq_f16 smaq 20 3 || exit $?
SMQ_BENCH_DTYPE=bf16 bash tools/profile_round.sh r3b_smaq_bf16 smaq 20 3 || exit $?
