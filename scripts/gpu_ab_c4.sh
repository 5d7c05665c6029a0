#!/bin/bash
# A/B of environment variants on the configs[4] sequence bench (ring-model prediction beside it)
# and align_chunk alone:  VARIANTS="base: fine:VGGT_GATE_FINE=1" bash scripts/gpu_ab_c4.sh TAG [config]
set -u
TAG=${1:-ab}
CFG=${2:-4}
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for v in ${VARIANTS:-base:}; do
  name=${v%%:*}
  envs=${v#*:}
  echo "[$(date +%T)] $name ($envs)"
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 240 python -u scripts/align_prof.py > "$OUT/align_$name.md" 2> "$OUT/align_$name.err" || exit 1
  tail -n 1 "$OUT/align_$name.md"
  env $(echo "$envs" | tr ',' ' ') VGGT_MFMA_PROBE=0 timeout -k 10 300 python -u bench.py --config "$CFG" --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/c${CFG}_$name.out" 2> "$OUT/c${CFG}_$name.err" || exit 1
  grep '^{' "$OUT/c${CFG}_$name.out" | tail -1 > "$OUT/c${CFG}_$name.json"
  python3 -c "
import json,sys; d=json.load(open('$OUT/c${CFG}_$name.json')); r=d['recurrence']; p=d['ring_model']['predicted']['8']
print(' ', d['ms_per_step'], 't_align', r['t_align_ms_under_load_median'], r['t_align_ms_alone_median'], 'T8', p['T_ms'], p['T1_over_TW'])"
done
echo "[$(date +%T)] done"
