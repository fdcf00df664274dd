#!/bin/bash
# Packed-compress kernel times (rocprofv3 kernel stats of bench.py --config packed) for the shipped
# library and each experiment build exp/<name>/libsmq.so given (tools/build_variant.py).
# Usage: bash tools/packed_exp.sh [variant names...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for v in shipped "$@"; do
  lib="$R/smart-quantization_amd/lib/libsmq.so"
  [ "$v" != shipped ] && lib="$R/exp/$v/libsmq.so"
  out="$R/gpurun_out/pexp_$v"
  SMQ_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out" -o run --output-format csv -- \
    python3 "$R/bench.py" --config packed --no-cpu-baseline --steps 10 --warmup 2 > "$out.log" 2>&1 || exit $?
  python3 - "$out/run_kernel_stats.csv" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "pack_block" in r["Name"]:
        print(sys.argv[2], r["Name"][:60], round(float(r["AverageNs"]) / 1000, 2), "us")
PY
done
