#!/bin/bash
# measurement experiment: packed bench with parts of the block kernel disabled (SMQ_PACK_EXP bits)
for e in 0 1 2 4 16 23; do
  echo "exp=$e"
  SMQ_PACK_EXP=$e bash tools/prof_trace.sh exp$e --config packed --steps 10 --warmup 2 | grep pack_block
done
