#!/bin/bash
# S2FP8 host path + packer check: the float / packed GPU tests, the S2FP8 host-cost breakdown, the
# s2fp8 and packed bench lines, a kernel trace of the packed config. Logs under gpurun_out/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_float.py tests/test_gpu_packed.py -m gpu > gpurun_out/t_s2pack.log 2>&1
rc=$?
tail -n 3 gpurun_out/t_s2pack.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/host_cost_s2.py > gpurun_out/host_cost_s2.log 2>&1 || exit $?
tail -n 1 gpurun_out/host_cost_s2.log
for c in s2fp8 packed; do
  timeout -k 10 240 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.json \
    2> gpurun_out/bench_$c.err || exit $?
  cut -c1-300 gpurun_out/bench_$c.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/s2pack_trace" -o run \
  --output-format csv -- python3 "$R/bench.py" --config packed --no-cpu-baseline --steps 20 \
  --warmup 3 > "$R/gpurun_out/s2pack_trace.log" 2>&1 || exit $?
grep -h 'pack\|stats' "$R"/gpurun_out/s2pack_trace/run_kernel_stats.csv | cut -c1-160
