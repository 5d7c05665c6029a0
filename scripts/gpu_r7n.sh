#!/bin/bash
# Tile-group height of the persistent GEMM (VGGT_GEMM_GM: M-panels per group in the XCD-aware tile order) with the
# round-3 loop, in the model.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  for g in 4 2 8 16; do
    VGGT_GEMM_GM=$g timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$OUT/gm$g.tmp" 2>> "$OUT/err.log" || exit $?
    cat "$OUT/gm$g.tmp" >> "$OUT/gm$g.json"
    echo "gm $g: $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" "$OUT/gm$g.tmp")"
  done
done
