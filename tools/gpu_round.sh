#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench. Each GPU step has its own time limit; stop at the
# first fault/abort/timeout (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" ; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    tests) step pytest_gpu 900 python -m pytest tests -m gpu -q -x -k "not slow" ;;
    tests_all) step pytest_gpu_all 1200 python -m pytest tests -m gpu -q ;;
    slow) step pytest_slow 600 python -m pytest tests -m "gpu and slow" -q ;;
    membench) step membench 300 ./tools/membench ;;
    statsbench) step statsbench 300 ./tools/statsbench ;;
    kbench) step kbench 300 python tools/kbench.py ;;
    rev) for r in 0 1; do SMQ_APPLY_REVERSE=$r step kbench_rev$r 300 python tools/kbench.py --quick; done ;;
    fqtiles) for v in 1 2; do SMQ_FQ_TILE=$v step bench_fp8_t$v 300 python bench.py --config fp8 --steps 50 --warmup 5; SMQ_FQ_TILE=$v step bench_s2fp8_t$v 300 python bench.py --config s2fp8 --steps 200 --warmup 20; done ;;
    cold) for v in 1 2; do SMQ_APPLY_TILE=$v step kbench_cold_t$v 300 python tools/kbench.py --quick --cold; done ;;
    chunks) for c in 4096 8192 16384 32768; do SMQ_MULTI_CHUNK=$c step bench_multi_c$c 300 python bench.py --config multi --steps 100 --warmup 10; done ;;
    statchunks) for c in 32768 65536 131072; do SMQ_MULTI_STATS_CHUNK=$c step bench_multi_s$c 300 python bench.py --config multi --steps 100 --warmup 10; done ;;
    diag) step bench_diag 300 python tools/bench_diag.py ;;
    warm) step bench_w3 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline &&
          step bench_w20 300 python bench.py --steps 50 --warmup 20 --no-cpu-baseline &&
          step bench_w50 300 python bench.py --steps 100 --warmup 50 --no-cpu-baseline ;;
    dist2) SMQ_BENCH_SHARE_DEVICE=1 SMQ_BENCH_BACKEND=gloo step bench_dist2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --elements 67108864 ;;
    tiles) for v in 1 2; do SMQ_APPLY_TILE=$v step kbench_tile$v 300 python tools/kbench.py --quick; done ;;
    profile) step profile 1500 bash tools/profile_round.sh ${ROUND:-r03} smaq ;;
    profile_*) c=${s#profile_}; step profile_$c 1500 bash tools/profile_round.sh ${ROUND:-r03}_$c $c 50 10 ;;
    bench_packed) step bench_packed 600 python bench.py --config packed --steps 20 --warmup 3 ;;
    bench_packed_single) SMQ_BENCH_PACK_FLAGS=2 step bench_packed_single 600 python bench.py --config packed --steps 20 --warmup 3 ;;
    tests_packed) step pytest_packed 600 python -u -m pytest tests/test_gpu_packed.py -x -q --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --steps 20 --warmup 3 --cpu-budget 8 ;;
    bench_cpu) step bench_cpu 300 python bench.py --config smaq_cpu --cpu-budget 5 ;;
    bench_all) step bench_fp8 300 python bench.py --config fp8 --steps 50 --warmup 5 &&
               step bench_s2fp8 300 python bench.py --config s2fp8 --steps 200 --warmup 20 &&
               step bench_multi 300 python bench.py --config multi --steps 100 --warmup 10 &&
               step bench_sampled 300 python bench.py --config smaq_sampled --steps 20 --warmup 3 --no-cpu-baseline &&
               step bench_packed 600 python bench.py --config packed --steps 20 --warmup 3 ;;
  esac
done
