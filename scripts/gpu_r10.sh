#!/bin/bash
# Round 5, alignment-step work: selected GPU tests, then align_chunk alone (scripts/align_prof.py)
# under kernel-variant A/Bs given as "NAME:ENV=V,ENV=V" words in $VARIANTS.
#   usage: VARIANTS="base: fused0:VGGT_FUSED_HEADNORM=0" TESTS="..." bash scripts/gpu_r10.sh TAG
set -u
TAG=${1:-r10}
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  echo "[$(date +%T)] pytest"
  timeout -k 10 600 python -u -m pytest $TESTS --maxfail=3 -v --timeout 300 --timeout-method thread \
    ${KEXPR:+-k "$KEXPR"} > "$OUT/pytest.out" 2> "$OUT/pytest.err" || { tail -n 30 "$OUT/pytest.out"; exit 1; }
  tail -n 2 "$OUT/pytest.out"
fi
for v in ${VARIANTS:-base:}; do
  name=${v%%:*}
  envs=${v#*:}
  echo "[$(date +%T)] align_prof $name ($envs)"
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 240 python -u scripts/align_prof.py > "$OUT/align_$name.md" 2> "$OUT/align_$name.err" || exit 1
  tail -n 1 "$OUT/align_$name.md"
done
if [ -n "${C3:-}" ]; then
  echo "[$(date +%T)] c3"
  env $(echo "$C3" | tr ',' ' ') timeout -k 10 400 python -u bench.py --config 3 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/c3.out" 2> "$OUT/c3.err" || exit 1
  grep '^{' "$OUT/c3.out" | tail -1 > "$OUT/c3.json"
fi
echo "[$(date +%T)] done"
