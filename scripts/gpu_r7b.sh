#!/bin/bash
# GEMM DMA-placement A/B (VGGT_GEMM_PIPE): bitwise check + kernel timings, then the aggregator step.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 python3 -u scripts/pipebench.py > "$OUT/pipebench.txt" 2>&1 || { tail -5 "$OUT/pipebench.txt"; exit 1; }
cat "$OUT/pipebench.txt"
for p in 0 3 1 2 0 3; do
  VGGT_GEMM_PIPE=$p timeout -k 10 200 python3 bench.py --no-cpu-baseline > "$OUT/agg_$p.json.tmp" 2>> "$OUT/err.log" || exit $?
  cat "$OUT/agg_$p.json.tmp" >> "$OUT/agg_$p.json"
  echo "pipe $p: $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" "$OUT/agg_$p.json.tmp")"
done
for a in 2 0 2 0; do
  VGGT_ATTN16=$a timeout -k 10 200 python3 bench.py --no-cpu-baseline > "$OUT/attn16_$a.json.tmp" 2>> "$OUT/err.log" || exit $?
  cat "$OUT/attn16_$a.json.tmp" >> "$OUT/attn16_$a.json"
  echo "attn16 $a: $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" "$OUT/attn16_$a.json.tmp")"
done
