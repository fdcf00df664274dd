#!/bin/bash
# Round-end check of the committed tree: the whole GPU suite, smoke(), the default bench line and
# the autograd (model-scale callers) line. Logs under gpurun_out/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/t_final.log 2>&1
rc=$?
tail -n 3 gpurun_out/t_final.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
timeout -k 10 240 python -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || exit $?
cut -c1-400 gpurun_out/final_bench.json
timeout -k 10 300 python -u bench.py --config autograd --no-cpu-baseline > gpurun_out/final_autograd.json \
  2> gpurun_out/final_autograd.err || exit $?
cut -c1-400 gpurun_out/final_autograd.json
