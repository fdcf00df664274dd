#!/bin/bash
# Round-5 final check at HEAD: the GPU suite, smoke, and a bench line of every config (no
# profiler), each step under its own limit, printing as it goes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG=${1:-r5i}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -n 30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
tail -n 1 gpurun_out/${TAG}_smoke.log
: > gpurun_out/${TAG}_bench.jsonl
timeout -k 10 300 python -u bench.py >> gpurun_out/${TAG}_bench.jsonl 2> gpurun_out/${TAG}_bench.err || exit 1
echo headline done
for c in multi packed s2fp8 fp8 autograd autograd_resnet34; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline >> gpurun_out/${TAG}_bench.jsonl \
    2>> gpurun_out/${TAG}_bench.err || exit 1
  echo $c done
done
for d in f16 bf16; do
  SMQ_BENCH_DTYPE=$d timeout -k 10 300 python -u bench.py --no-cpu-baseline >> gpurun_out/${TAG}_bench.jsonl \
    2>> gpurun_out/${TAG}_bench.err || exit 1
  echo $d done
done
echo done
