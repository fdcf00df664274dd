#!/bin/bash
# Half-input apply study: kernel traces (f32 / f16 / bf16) and one SQ pass each for f32 and f16.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
SMQ_BENCH_DTYPE=f16 bash "$R/tools/prof_trace.sh" h16 --steps 20 --warmup 3 &&
SMQ_BENCH_DTYPE=bf16 bash "$R/tools/prof_trace.sh" hb16 --steps 20 --warmup 3 &&
bash "$R/tools/prof_trace.sh" h32 --steps 20 --warmup 3 &&
SMQ_BENCH_DTYPE=f16 bash "$R/tools/prof_pmc.sh" h16 "$C" --steps 5 --warmup 2 &&
bash "$R/tools/prof_pmc.sh" h32 "$C" --steps 5 --warmup 2
