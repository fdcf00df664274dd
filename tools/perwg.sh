R=$GRAFT_REPO_ROOT
for w in 8192 32768 65536 131072; do
  SMQ_STATS_PER_WG=$w timeout -k 10 300 python $R/bench.py --config autograd --steps 20 --warmup 3 > $R/gpurun_out/perwg_$w.log 2>&1 || exit $?
done
