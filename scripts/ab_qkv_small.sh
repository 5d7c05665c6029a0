#!/bin/bash
# qkv / fc1 ping-pong tile width at short M (6,592 rows) and the chunk shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${1:-ab_qkv}
mkdir -p "$OUT"
for r in 1 2; do
  timeout -k 10 300 python -u scripts/kbench.py --only gemm --gemm-modes 4,5,6,7,0 --reps 40 --tokens 6592 > "$OUT/m6592_$r.log" 2>&1 || exit $?
done
timeout -k 10 300 python -u scripts/kbench.py --only gemm --gemm-modes 4,7 --reps 30 > "$OUT/m21984.log" 2>&1 || exit $?
grep -h -E "^(qkv|fc1|qkv_fused)" "$OUT"/*.log
