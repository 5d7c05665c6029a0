#!/bin/bash
# Fused residual-add/LayerNorm default (3) vs the RMW epilogues (0) on the chunk and sequence workloads.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
bash scripts/ab_combo.sh $1_c4 "VGGT_FUSED_ADD_LN=0 VGGT_FUSED_ADD_LN=3" 2 --workload sequence --seq-frames 512 --height 154 --steps 2 --warmup 1 || exit $?
bash scripts/ab_combo.sh $1_chunk "VGGT_FUSED_ADD_LN=0 VGGT_FUSED_ADD_LN=3" 2 --workload chunk --steps 4 --warmup 2 || exit $?
bash scripts/ab_combo.sh $1_c3 "VGGT_FUSED_ADD_LN=0 VGGT_FUSED_ADD_LN=3" 2 --workload sequence --seq-frames 64 --steps 2 --warmup 1 || exit $?
