#!/bin/bash
# Re-entry check at HEAD on a fresh build: the GPU suite, smoke and the default bench line.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5t}
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -n 2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
tail -n 1 gpurun_out/${T}_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.jsonl 2> gpurun_out/${T}_bench.err || exit 1
cut -c1-400 gpurun_out/${T}_bench.jsonl
timeout -k 10 400 python -u tools/saved_ab.py 3 > gpurun_out/${T}_saved_ab.txt 2>&1 || { tail -n 20 gpurun_out/${T}_saved_ab.txt; exit 1; }
head -n 4 gpurun_out/${T}_saved_ab.txt
echo done
