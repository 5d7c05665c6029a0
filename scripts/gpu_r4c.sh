#!/bin/bash
# Parity of the fused residual/LayerNorm default + the 128x128 residual prefetch, then A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_aggregator.py tests/test_gpu_model.py tests/test_gpu_kernels.py -k "gemm or aggregator or model or resid" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for e in 0 1; do VGGT_GEMM_RPF=$e timeout -k 10 300 python scripts/gemmbench.py --modes=-1 --shapes proj,fc2 --epis plain,resid > "$OUT/gemm_rpf$e.log" 2>&1 || exit $?; grep -v '^{' "$OUT/gemm_rpf$e.log" | sed "s/^/rpf=$e /"; done
bash scripts/ab_combo.sh $1 "VGGT_FUSED_ADD_LN=1,VGGT_GEMM_RPF=0 VGGT_FUSED_ADD_LN=1,VGGT_GEMM_RPF=1 VGGT_FUSED_ADD_LN=3,VGGT_GEMM_RPF=0" 3 --steps 5 --warmup 2
