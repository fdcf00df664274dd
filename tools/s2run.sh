#!/bin/bash
# S2FP8 GPU session: tests of the S2FP8 paths, graph-safe tests, the per-workgroup trace, s2bench
# and the C4 bench line. Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 4 | cut -c1-1500
  [ $rc -eq 0 ] || exit $rc
}
run s2_tests 300 python -u -m pytest tests/test_gpu_float.py -x -q --timeout 120 --timeout-method thread -k s2fp8
run s2_graph 300 python -u -m pytest tests/test_gpu_graph_safe.py -x -q --timeout 120 --timeout-method thread
run s2trace 120 python tools/s2trace.py
run s2bench 120 python tools/s2bench.py
run bench_s2 120 python bench.py --config s2fp8 --steps 200 --warmup 20
if [ -n "$S2_LDS_SWEEP" ]; then
  for kb in 0 48; do
    SMQ_S2_LDS_KB=$kb run s2trace_lds$kb 120 python tools/s2trace.py
    SMQ_S2_LDS_KB=$kb run s2bench_lds$kb 120 python tools/s2bench.py
  done
fi
