#!/bin/bash
# Round-3 check: fp64 / large-k / half-input GPU tests, then fp16 / bf16 traces of the bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_f64.py tests/test_gpu_sampled.py tests/test_gpu_smaq.py -m "gpu and not slow" \
  > gpurun_out/t_r3b.log 2>&1
rc=$?
tail -n 5 gpurun_out/t_r3b.log
[ $rc -eq 0 ] || exit $rc
SMQ_BENCH_DTYPE=f16 bash tools/prof_trace.sh h16b --steps 20 --warmup 3 &&
SMQ_BENCH_DTYPE=bf16 bash tools/prof_trace.sh hb16b --steps 20 --warmup 3
