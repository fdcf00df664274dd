#!/bin/bash
# Whole GPU suite, then the default bench line and every config's line. Logs under gpurun_out/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/t_full.log 2>&1
rc=$?
tail -n 5 gpurun_out/t_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
cat gpurun_out/bench_default.json
for c in ${BENCH_CONFIGS:-fp8 s2fp8 multi packed}; do
  timeout -k 10 240 python -u bench.py --config "$c" --no-cpu-baseline >> gpurun_out/bench_configs.jsonl \
    2> "gpurun_out/bench_$c.err" || exit $?
done
cut -c1-400 gpurun_out/bench_configs.jsonl
