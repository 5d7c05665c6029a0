#!/bin/bash
# 16x16 attention accuracy vs the 32x32 form, and the full-model training-gradient test under both forms.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${1:-r6e}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "attention16" > "$OUT/acc.log" 2>&1; echo "acc rc=$?"
grep "rel-L2\|passed\|failed" "$OUT/acc.log"
for m in 0 1; do
  VGGT_ATTN16=$m timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py -k "feature_aligned_training_step or two_chunk" > "$OUT/train_$m.log" 2>&1; echo "train ATTN16=$m rc=$?"
  grep "worst\|passed\|failed" "$OUT/train_$m.log" | cut -c1-400
done
