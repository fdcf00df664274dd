#!/bin/bash
# Round-5 evidence on one box: the GPU suite, smoke, a bench line of every config, then a kernel
# trace + FETCH / WRITE passes per profiled config (tools/profile_round.sh; summarised on the host
# by tools/pmc_traffic.py / tools/autograd_profile.py into profiles/<tag>_*) and the single-launch
# SmaQ at 1M / 4M / 8M (tools/profile_fused.sh). Each step under its own time limit; the first
# failure ends the script.
# Usage: bash tools/gpu_round5.sh <tag>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG=${1:-r5a}
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -n 30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -n 2 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
tail -n 1 gpurun_out/${TAG}_smoke.log
: > gpurun_out/${TAG}_bench.jsonl
timeout -k 10 300 python -u bench.py >> gpurun_out/${TAG}_bench.jsonl 2> gpurun_out/${TAG}_bench.err || exit 1
for c in multi packed s2fp8 fp8 autograd autograd_resnet34; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline >> gpurun_out/${TAG}_bench.jsonl \
    2>> gpurun_out/${TAG}_bench.err || exit 1
done
for d in f16 bf16; do
  SMQ_BENCH_DTYPE=$d timeout -k 10 300 python -u bench.py --no-cpu-baseline >> gpurun_out/${TAG}_bench.jsonl \
    2>> gpurun_out/${TAG}_bench.err || exit 1
done
for c in smaq multi packed s2fp8 fp8 autograd_resnet34; do
  bash tools/profile_round.sh ${TAG}_$c $c > /dev/null || exit 1
done
# the autograd trace and counter files are large (thousands of dispatches with long names): keep the
# per-size-class summary (tools/autograd_profile.py) and the stats, drop the raw CSVs
AG=gpurun_out/prof_${TAG}_autograd_resnet34
python tools/autograd_profile.py $AG gpurun_out/${TAG}_autograd_resnet34_summary.json > /dev/null || exit 1
rm -f $AG/trace/run_kernel_trace.csv $AG/fetch/run_counter_collection.csv $AG/write/run_counter_collection.csv
SMQ_BENCH_DTYPE=f16 bash tools/profile_round.sh ${TAG}_smaq_f16 smaq > /dev/null || exit 1
SMQ_BENCH_DTYPE=bf16 bash tools/profile_round.sh ${TAG}_smaq_bf16 smaq > /dev/null || exit 1
bash tools/profile_fused.sh ${TAG}_fused > /dev/null || exit 1
du -sh gpurun_out
echo done
