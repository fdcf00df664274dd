cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in 8192 32768; do
  SMQ_MULTI_CHUNK=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/chunk_$c -o run --output-format csv -- python3 $R/bench.py --config multi --steps 30 --warmup 3 > $R/gpurun_out/chunk_$c.log 2>&1 || exit $?
done
