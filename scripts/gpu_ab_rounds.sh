#!/bin/bash
# Same-box interleaved A/B of the round-4 tree (ab_r4/, git archive of 83683b2, built in place) against this
# tree: the headline (configs[1]) and configs[3].   usage: bash scripts/gpu_ab_rounds.sh TAG
set -u
TAG=${1:-abr}
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in 1 2 3; do
  for t in r4 r5; do
    B=bench.py; [ $t = r4 ] && B=ab_r4/bench.py
    VGGT_MFMA_PROBE=0 timeout -k 10 200 python -u $B --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/head_${t}_$r.out" 2>&1 || exit 1
    grep '^{' "$OUT/head_${t}_$r.out" | tail -1 > "$OUT/head_${t}_$r.json"
    python3 -c "import json; d=json.load(open('$OUT/head_${t}_$r.json')); print('head', '$t', $r, d['ms_per_step'])"
  done
done
for r in 1 2; do
  for t in r4 r5; do
    B=bench.py; [ $t = r4 ] && B=ab_r4/bench.py
    VGGT_RECURRENCE_PROBE=0 timeout -k 10 300 python -u $B --config 3 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/c3_${t}_$r.out" 2>&1 || exit 1
    grep '^{' "$OUT/c3_${t}_$r.out" | tail -1 > "$OUT/c3_${t}_$r.json"
    python3 -c "import json; d=json.load(open('$OUT/c3_${t}_$r.json')); print('c3', '$t', $r, d['ms_per_step'])"
  done
done
echo done
