#!/bin/bash
# The packed-saved / ratio-logging ResNet-34 step: the saved-activation GPU tests, two bench lines
# of --config autograd_resnet34, then a kernel trace of the packed-saved step summarised per kernel
# (tools/kernel_summary.py) and the interleaved A/B of tools/saved_ab.py.
# Usage: bash tools/gpu_saved_step.sh <tag>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
T=${1:-saved}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_saved.py tests/test_gpu_roundtrip_compress.py > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_bench.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config autograd_resnet34 --no-cpu-baseline >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || { tail -n 20 gpurun_out/${T}_bench.err; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/${T}_bench.jsonl'):
    d=json.loads(l); v=d['variants']
    print({k: (v[k]['ms_per_step'], v[k].get('vs_smaq_eager'), (v[k].get('memory') or {}).get('step_peak_above_resident_mib')) for k in v})
"
timeout -k 10 400 python -u tools/saved_ab.py 5 > gpurun_out/${T}_saved_ab.txt 2>&1 || { tail -n 20 gpurun_out/${T}_saved_ab.txt; exit 1; }
head -n 3 gpurun_out/${T}_saved_ab.txt | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${T}_saved" -o run --output-format csv -- python3 "$R/tools/saved_trace.py" 10 packed > "$R/gpurun_out/${T}_saved_trace.log" 2>&1 || { tail -n 20 "$R/gpurun_out/${T}_saved_trace.log"; exit 1; }
python3 "$R/tools/kernel_summary.py" "$R/gpurun_out/prof_${T}_saved" "$R/gpurun_out/${T}_saved_kernels.json" 13 "ResNet-34 CIFAR b128 step with PackedActivations, 13 steps under rocprofv3 --kernel-trace (tools/saved_trace.py 10)"
rm -f "$R"/gpurun_out/prof_${T}_saved/run_kernel_trace.csv
echo done
