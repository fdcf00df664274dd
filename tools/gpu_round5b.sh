#!/bin/bash
# Round-5 evidence at the session's final code: the GPU suite, smoke, the headline and the packed /
# autograd bench lines, rocprofv3 kernel traces + FETCH / WRITE passes of packed and the ResNet-34
# autograd config (per-size-class summary), and the packed-saved step's kernel trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG=${1:-r5h}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -n 30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -n 2 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
tail -n 1 gpurun_out/${TAG}_smoke.log
: > gpurun_out/${TAG}_bench.jsonl
timeout -k 10 300 python -u bench.py >> gpurun_out/${TAG}_bench.jsonl 2> gpurun_out/${TAG}_bench.err || exit 1
for c in packed autograd_resnet34; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline >> gpurun_out/${TAG}_bench.jsonl \
    2>> gpurun_out/${TAG}_bench.err || exit 1
done
for c in packed autograd_resnet34; do
  bash tools/profile_round.sh ${TAG}_$c $c > /dev/null || exit 1
done
AG=gpurun_out/prof_${TAG}_autograd_resnet34
python tools/autograd_profile.py $AG gpurun_out/${TAG}_autograd_resnet34_summary.json > /dev/null || exit 1
rm -f $AG/trace/run_kernel_trace.csv $AG/fetch/run_counter_collection.csv $AG/write/run_counter_collection.csv
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_saved" -o run --output-format csv -- python3 "$R/tools/saved_trace.py" 10 packed > "$R/gpurun_out/${TAG}_saved_trace.log" 2>&1 || exit 1
cd "$R"
du -sh gpurun_out
echo done
