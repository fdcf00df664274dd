set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_hostpath.py tests/test_gpu_optim.py > gpurun_out/r5b_tests.log 2>&1 || { tail -n 40 gpurun_out/r5b_tests.log; exit 1; }
tail -n 2 gpurun_out/r5b_tests.log
timeout -k 10 200 python -u tools/host_cost_smaq.py > gpurun_out/r5b_hc_smaq.txt 2>&1 || { tail -20 gpurun_out/r5b_hc_smaq.txt; exit 1; }
head -3 gpurun_out/r5b_hc_smaq.txt
: > gpurun_out/r5b_bench.jsonl
for c in autograd_resnet34 autograd s2fp8; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline >> gpurun_out/r5b_bench.jsonl 2>> gpurun_out/r5b_bench.err || exit 1
done
echo done
