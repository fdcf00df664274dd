#!/bin/bash
# Apply-path check after a change to the element chain: the SmaQ GPU tests, then per dtype a kernel
# trace and an SQ_INSTS_VALU pass of the headline bench. Logs under gpurun_out/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  ${PAIR_TESTS:-tests/test_gpu_smaq.py tests/test_gpu_multi.py tests/test_gpu_graph_safe.py} -m gpu \
  > gpurun_out/t_pair.log 2>&1
rc=$?
tail -n 5 gpurun_out/t_pair.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for dt in ${PAIR_DTYPES:-f32 f16 bf16}; do
  [ "$dt" = f32 ] && E="" || E="$dt"
  OUT="$R/gpurun_out/pair_$dt"; mkdir -p "$OUT"
  SMQ_BENCH_DTYPE=$E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run \
    --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 20 --warmup 3 \
    > "$OUT/trace.log" 2>&1 || exit $?
  SMQ_BENCH_DTYPE=$E timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE \
    -d "$OUT/pmc" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline \
    --steps 3 --warmup 1 > "$OUT/pmc.log" 2>&1 || exit $?
  grep -h 'smaq_apply\|smaq_stats' "$OUT"/trace/*/run_kernel_stats.csv "$OUT"/trace/run_kernel_stats.csv 2>/dev/null | cut -c1-200
  grep '"metric"' "$OUT/trace.log" | cut -c1-200
done
