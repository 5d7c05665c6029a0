#!/bin/bash
# 4- vs 8-wave attention workgroups at 21,984 / 10,992 / 6,592 tokens (kbench, alternating rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${1:-ab_w8}
mkdir -p "$OUT"
for T in 21984 10992 6592; do
  timeout -k 10 300 python -u scripts/kbench.py --only attn --attn-waves 4,8 --attn-variants 33 --rounds 3 --tokens $T > "$OUT/m$T.log" 2>&1 || exit $?
done
grep -h "^global_attn\|^frame_attn" "$OUT"/m*.log
