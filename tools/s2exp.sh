set -e
SMQ_S2_LAST=1 timeout -k 10 300 python -m pytest tests/test_gpu_float.py -x -q -k s2fp8 > gpurun_out/s2last_tests.log 2>&1 || { tail -20 gpurun_out/s2last_tests.log; exit 1; }
tail -1 gpurun_out/s2last_tests.log
for last in 0 1; do
  echo "== last=$last"
  SMQ_S2_LAST=$last bash tools/ktrace.sh s2_last$last s2fp8 300 | grep -v rocprofv3 | cut -c1-200
  SMQ_S2_LAST=$last timeout -k 10 120 python bench.py --config s2fp8 --steps 300 --warmup 20 | cut -c1-200
done
