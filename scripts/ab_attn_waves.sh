#!/bin/bash
# Attention workgroup size (2 / 4 / 8 waves) at the chunk shape and at the
# 154x518 sequence shape (6,592 tokens), after the attention tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${1:-ab_attn}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "attention" > "$OUT/pytest_attn.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_attn.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/kbench.py --only attn --attn-waves 4,2,8 --attn-variants 33 --rounds 2 --tokens 6592 > "$OUT/m6592.log" 2>&1 || exit $?
timeout -k 10 300 python -u scripts/kbench.py --only attn --attn-waves 4,2 --attn-variants 33 --rounds 2 > "$OUT/m21984.log" 2>&1 || exit $?
grep -h "attn" "$OUT"/m*.log
