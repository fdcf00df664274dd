#!/bin/bash
# A/B: packer blocks in address order vs reverse order (knobs build).
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5n}
bash tools/ab_env.sh 4 "--config packed" "SMQ_PACK_FORWARD=0" "SMQ_PACK_FORWARD=1" > gpurun_out/${T}_ab.txt 2>&1 || exit 1
cat gpurun_out/${T}_ab.txt
