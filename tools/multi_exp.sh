#!/bin/bash
# Multi-tensor kernel times of the C5 bench (rocprofv3 kernel stats) for the shipped library, then
# each variant given: a name = exp/<name>/libsmq.so (tools/build_variant.py <name> -D...), or
# KNOB=VALUE = the knob build (exp/knobs, -DSMQ_KNOBS=1) with that environment setting.
# Usage: bash tools/multi_exp.sh [variant | KNOB=VALUE ...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for v in shipped "$@"; do
  lib="$R/smart-quantization_amd/lib/libsmq.so"; knob=""
  case "$v" in
    shipped) ;;
    *=*) lib="$R/exp/knobs/libsmq.so"; knob="$v" ;;
    *) lib="$R/exp/$v/libsmq.so" ;;
  esac
  out="$R/gpurun_out/mexp_${v//=/_}"
  env $knob SMQ_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out" -o run --output-format csv -- \
    python3 "$R/bench.py" --config multi --no-cpu-baseline --steps 20 > "$out.log" 2>&1 || exit $?
  python3 - "$out/run_kernel_stats.csv" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "smaq_multi" in r["Name"]:
        print(sys.argv[2], r["Name"][:48], round(float(r["AverageNs"]) / 1000, 2), "us")
PY
done
