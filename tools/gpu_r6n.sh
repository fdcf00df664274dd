#!/bin/bash
# Single-launch packer (look-back) for activation sizes: packed / saved / roundtrip-compress GPU
# tests, the saved-mode A/B and kernel trace, and the 256M packed bench + its kernel trace (the var
# kernel's inlined re-code).
set -o pipefail
mkdir -p gpurun_out
T=${1:-r6n}
R="${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_saved.py tests/test_gpu_roundtrip_compress.py tests/test_gpu_packed.py tests/test_gpu_graph_safe.py tests/test_gpu_optim.py tests/test_packed_f64.py tests/test_gpu_workspace.py > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
timeout -k 10 400 python -u tools/saved_ab.py 5 > gpurun_out/${T}_saved_ab.txt 2>&1 || { tail -n 20 gpurun_out/${T}_saved_ab.txt; exit 1; }
head -n 5 gpurun_out/${T}_saved_ab.txt | cut -c1-300
: > gpurun_out/${T}_packed_bench.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config packed --no-cpu-baseline >> gpurun_out/${T}_packed_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/${T}_packed_bench.jsonl'):
    d=json.loads(l); print(d['config'].get('workload'), d['ms_per_step'], d.get('compress_ms'), d.get('decompress_ms'))
"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${T}_saved" -o run --output-format csv -- python3 "$R/tools/saved_trace.py" 10 packed > "$R/gpurun_out/${T}_saved_trace.log" 2>&1 || { tail -n 20 "$R/gpurun_out/${T}_saved_trace.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${T}_packed" -o run --output-format csv -- python3 "$R/bench.py" --config packed --no-cpu-baseline --steps 20 --warmup 3 > "$R/gpurun_out/${T}_packed_trace.log" 2>&1 || { tail -n 20 "$R/gpurun_out/${T}_packed_trace.log"; exit 1; }
rm -f "$R"/gpurun_out/prof_${T}_packed/run_kernel_trace.csv
echo done
