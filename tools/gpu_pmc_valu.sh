#!/bin/bash
# VALU / wave-cycle counters of the headline apply (fp32, fp16) and the packer, plus the S2FP8 host
# cost breakdown. Logs under gpurun_out/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/host_cost_s2.py > gpurun_out/host_cost_s2.log 2>&1 || exit $?
cat gpurun_out/host_cost_s2.log
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
bash tools/pmc_passes.sh valu_f32 smaq "$C" || exit $?
SMQ_BENCH_DTYPE=f16 bash tools/pmc_passes.sh valu_f16 smaq "$C" || exit $?
bash tools/pmc_passes.sh valu_packed packed "$C" || exit $?
