cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for gcap in 512 1024 1536 2048; do
  SMQ_STATS_GRID=$gcap timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/sg_$gcap -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/sg_$gcap.log 2>&1 || exit $?
done
