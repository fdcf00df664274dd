#!/bin/bash
# Experiment: the one-launch (look-back) packer at every size (exp/lb_all, -DSMQ_LB_MAX_BLOCKS=1048576)
# against the shipped build (one launch up to 2048 blocks, three above): packed tests on the
# variant, then interleaved 256M packed bench lines and a kernel trace of the variant.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r6l}
R="${GRAFT_REPO_ROOT:-$(pwd)}"
V="$R/exp/lb_all/libsmq.so"
SMQ_LIB=$V timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_packed.py tests/test_gpu_roundtrip_compress.py > gpurun_out/${T}_tests.log 2>&1 || { tail -n 30 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_ab.jsonl
for i in 1 2 3; do
  for lib in shipped variant; do
    if [ $lib = variant ]; then export SMQ_LIB=$V; else unset SMQ_LIB; fi
    timeout -k 10 300 python -u bench.py --config packed --no-cpu-baseline > gpurun_out/${T}_one.json 2>> gpurun_out/${T}_bench.err || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/${T}_one.json')); print('$lib', d['ms_per_step'], d.get('compress_ms'), d.get('decompress_ms'))" | tee -a gpurun_out/${T}_ab.txt
  done
done
unset SMQ_LIB
cd /tmp && export TMPDIR=/tmp
SMQ_LIB=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${T}_variant" -o run --output-format csv -- python3 "$R/bench.py" --config packed --no-cpu-baseline --steps 20 --warmup 3 > "$R/gpurun_out/${T}_trace.log" 2>&1 || exit 1
rm -f "$R"/gpurun_out/prof_${T}_variant/run_kernel_trace.csv
echo done
