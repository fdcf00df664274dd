#!/bin/bash
# Saved-activation mode after routing grad-map calls through SmartFP and asynchronous size checks:
# its GPU tests, the A/B and a kernel trace of the packed step (per-dispatch trace kept).
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5v}
R="${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_saved.py tests/test_gpu_roundtrip_compress.py tests/test_gpu_packed.py tests/test_gpu_graph_safe.py > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
timeout -k 10 400 python -u tools/saved_ab.py 5 > gpurun_out/${T}_saved_ab.txt 2>&1 || { tail -n 20 gpurun_out/${T}_saved_ab.txt; exit 1; }
head -n 5 gpurun_out/${T}_saved_ab.txt | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${T}_saved" -o run --output-format csv -- python3 "$R/tools/saved_trace.py" 10 packed > "$R/gpurun_out/${T}_saved_trace.log" 2>&1 || { tail -n 20 "$R/gpurun_out/${T}_saved_trace.log"; exit 1; }
echo done
