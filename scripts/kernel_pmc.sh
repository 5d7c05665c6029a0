#!/bin/bash
# SQ anatomy passes (one rocprofv3 --pmc run per counter group) over one command,
# summarised on the box by scripts/pmc_anatomy.py.   usage: TAG KERNEL CMD...
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
KERN=$2
shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
P=/tmp/pmc_$(basename "$OUT")
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $P/p1 -o run -- "$@" > "$OUT/p1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $P/p2 -o run -- "$@" > "$OUT/p2.log" 2>&1 || exit $?
python3 scripts/pmc_anatomy.py $P/p1 $P/p2 --kernel "$KERN" ${GRID:+--grid $GRID} --out "$OUT/anatomy.md"
