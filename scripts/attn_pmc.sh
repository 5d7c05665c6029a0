#!/bin/bash
# PMC anatomy of the global-attention kernel (kbench attention, production variant 33):
# issue / wait breakdown and MFMA busy cycles, one rocprofv3 pass per counter group.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${1:-attn_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python3 scripts/kbench.py --only attn --attn-waves 4 --attn-variants 33 --reps 8 --warm-s 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/p1" -o run -- $CMD > "$OUT/p1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS -d "$OUT/p2" -o run -- $CMD > "$OUT/p2.log" 2>&1 || exit $?
echo done
