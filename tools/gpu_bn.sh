# Packed BN / negative-threshold support: the packed and smaq GPU tests, then the packed bench
# (the default decoder's VGPRs went 67 -> 71, same 7 waves per SIMD: check the round trip).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_packed.py tests/test_gpu_smaq.py -m gpu > gpurun_out/t_bn.log 2>&1; rc=$?; tail -3 gpurun_out/t_bn.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do timeout -k 10 180 python bench.py --config packed --steps 20 2>/dev/null | tail -1 | cut -c1-200 >> gpurun_out/bn_packed_bench.txt || exit 1; done
cat gpurun_out/bn_packed_bench.txt
