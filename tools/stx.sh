# persistent apply A/B on the headline bench (interleaved, 3 rounds)
SMQ_APPLY_PERSIST=1024 timeout -k 10 300 python -m pytest tests/test_gpu_smaq.py tests/test_gpu_graph_safe.py -x -q > gpurun_out/stx_tests.log 2>&1; rc=$?; tail -1 gpurun_out/stx_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
for g in 0 512 1024 1536 2048; do
  printf "persist=%s " $g
  SMQ_APPLY_PERSIST=$g timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done; done
