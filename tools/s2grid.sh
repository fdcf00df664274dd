cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for gcap in 96 192 384 768; do
  SMQ_S2_STATS_GRID=$gcap timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s2g_$gcap -o run --output-format csv -- python3 $R/bench.py --config s2fp8 --steps 100 --warmup 10 > $R/gpurun_out/s2g_$gcap.log 2>&1 || exit $?
done
