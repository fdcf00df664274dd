#!/bin/bash
# Round-2 closing evidence: profiles (kernel trace + FETCH/WRITE passes) of every config, then the
# bench lines. Stops at the first fault / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in smaq s2fp8 packed fp8 multi smaq_sampled; do
  if [ $c = smaq ]; then tag=r2c; else tag=r2c_$c; fi
  timeout -k 10 900 bash tools/profile_round.sh $tag $c 20 5 > gpurun_out/pr_$c.log 2>&1 || { echo "profile $c failed"; exit 1; }
  echo "profiled $c"
done
timeout -k 10 600 bash tools/ktrace.sh r2c_autograd autograd 20 > gpurun_out/pr_autograd.log 2>&1 || exit 1
echo profiled autograd
