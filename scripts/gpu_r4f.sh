#!/bin/bash
# Single-slot attention (variant 161): parity, kernel A/B vs 33 at the frame / global shapes, in-model A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "attention" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python scripts/kbench.py --only attn --attn-variants 33,161 --attn-waves 4,8 --rounds 3 > "$OUT/kbench.log" 2>&1 || exit $?
grep -v '^{' "$OUT/kbench.log"
bash scripts/ab_env.sh $1 VGGT_ATTN_VARIANT "33 161" 2 --steps 5 --warmup 2
