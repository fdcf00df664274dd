# packed codec: GPU tests, then kernel trace of the packed bench config
timeout -k 10 300 python -u -m pytest tests/test_gpu_packed.py tests/test_gpu_smaq.py -x -q --timeout 120 --timeout-method thread -k "not slow" > gpurun_out/packed_tests.log 2>&1; rc=$?
tail -3 gpurun_out/packed_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/packed_tests.log | head -20; exit $rc; }
bash tools/ktrace.sh pk packed 20 | grep -v rocprofv3
