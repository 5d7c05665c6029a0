#!/bin/bash
# one lease: CU-mask probe + non-persistent recurrence probe, interleaved ATTN16 A/B of
# the headline, then the round-4 kernel-trace / DPT-traffic profiles
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
T=${1:-r8l}
bash scripts/gpu_cumask.sh $T || exit $?
OUT=gpurun_out/$T
for i in 1 2 3; do
  for a in 2 1; do
    timeout -k 10 200 env VGGT_ATTN16=$a python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/ab_attn16_${a}_$i.out" 2>&1 || exit $?
    echo "attn16=$a run $i: $(grep '^{' "$OUT/ab_attn16_${a}_$i.out" | tail -1 | cut -c1-160)"
  done
done
bash scripts/gpu_prof_r8.sh $T || exit $?
echo all done
