#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do timeout -k 10 120 ./tools/launch_cost >> gpurun_out/r5s_launch_cost.txt 2>&1 || exit 1; done
cat gpurun_out/r5s_launch_cost.txt
