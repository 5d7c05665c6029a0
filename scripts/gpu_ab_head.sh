#!/bin/bash
# Interleaved A/B of environment variants on the headline bench (configs[1]):
#   VARIANTS="base: split4:VGGT_ATTN_SPLIT=4" ROUNDS=2 bash scripts/gpu_ab_head.sh TAG
set -u
TAG=${1:-abh}
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for v in ${VARIANTS:-base:}; do
    name=${v%%:*}
    envs=${v#*:}
    env $(echo "$envs" | tr ',' ' ') VGGT_MFMA_PROBE=0 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/head_${name}_$r.out" 2> "$OUT/head_${name}_$r.err" || exit 1
    grep '^{' "$OUT/head_${name}_$r.out" | tail -1 > "$OUT/head_${name}_$r.json"
    python3 -c "
import json; d=json.load(open('$OUT/head_${name}_$r.json')); print('$name', $r, d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  done
done
echo "[$(date +%T)] done"
