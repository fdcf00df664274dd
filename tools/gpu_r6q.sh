set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_roundtrip_compress.py tests/test_gpu_saved.py tests/test_gpu_hostpath.py tests/test_saved_notify.py > gpurun_out/r6q_tests.txt 2>&1 && tail -3 gpurun_out/r6q_tests.txt && \
timeout -k 10 500 python -u tools/saved_ab.py 5 smartfp,packed,packed_event > gpurun_out/r6q_ab.txt 2>&1 ; grep -a "ms/step\|peak\|passed\|failed" gpurun_out/r6q_ab.txt gpurun_out/r6q_tests.txt | cut -c1-400
