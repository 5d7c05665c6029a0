#!/bin/bash
# 16x16x32 attention variant (161): parity tests, then A/B vs 33 at the global / sequence shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${1:-r6c}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "attention" > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for T in 21984 6592; do
  timeout -k 10 300 python -u scripts/kbench.py --only attn --attn-waves 4,8 --attn-variants 33,161 --rounds 3 --tokens $T > "$OUT/ab$T.log" 2>&1 || exit $?
done
grep -h "^global_attn" "$OUT"/ab*.log
