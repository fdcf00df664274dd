set -o pipefail
SMQ_LIB=$PWD/exp/dec2/libsmq.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_packed.py -m gpu > gpurun_out/t_dec2.log 2>&1; rc=$?; tail -3 gpurun_out/t_dec2.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_lib.sh $PWD/smart-quantization_amd/lib/libsmq.so $PWD/exp/dec2/libsmq.so 3 "packed||--config packed --steps 20" > gpurun_out/ab_dec2.txt 2>&1; rc=$?; cat gpurun_out/ab_dec2.txt; exit $rc
