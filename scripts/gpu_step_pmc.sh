#!/bin/bash
# Counter passes over one aggregator bench step -> profiles-ready step_mfma.json
#   usage: bash scripts/gpu_step_pmc.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline"
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/spmc/busy -o run -- $BENCH > "$OUT/busy.log" 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE --output-format csv -d /tmp/spmc/mops -o run -- $BENCH > "$OUT/mops.log" 2>&1 || echo "mops pass failed (counter unavailable?)"
python3 scripts/step_pmc.py /tmp/spmc/busy $( [ -d /tmp/spmc/mops ] && echo /tmp/spmc/mops ) --out "$OUT/step_mfma.json"
