#!/bin/bash
# Packed-saved step kernel trace (packed and SmartFP), the statistics launch of the packed
# compress in four modes (tools/packed_stats_ab.py), each under rocprofv3 --kernel-trace --stats.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r5u}
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
for k in packed_exit smartfp; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${T}_saved_$k" -o run --output-format csv -- python3 "$R/tools/saved_trace.py" 10 $k > "$R/gpurun_out/${T}_saved_$k.log" 2>&1 || { tail -n 20 "$R/gpurun_out/${T}_saved_$k.log"; exit 1; }
  tail -n 1 "$R/gpurun_out/${T}_saved_$k.log" | cut -c1-300
done
for m in roundtrip compress packed packed_nt; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${T}_pstats_$m" -o run --output-format csv -- python3 "$R/tools/packed_stats_ab.py" $m 30 > "$R/gpurun_out/${T}_pstats_$m.log" 2>&1 || { tail -n 20 "$R/gpurun_out/${T}_pstats_$m.log"; exit 1; }
  tail -n 1 "$R/gpurun_out/${T}_pstats_$m.log"
done
cd "$R"
rm -f gpurun_out/prof_${T}_*/run_kernel_trace.csv
echo done
