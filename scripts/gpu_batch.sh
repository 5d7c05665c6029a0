#!/bin/bash
# One GPU lease, several measurements: parity tests first, then bench lines
# (each step under its own time limit; the chain stops at the first failure).
#   usage: bash scripts/gpu_batch.sh TAG [tests|benches|all]
set -u
TAG=${1:-batch}
WHAT=${2:-all}
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  tail -n 2 "$OUT/$name.out"
  return $rc
}
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  step pytest 1000 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_ring.py tests/test_gpu_align.py tests/test_gpu_small_kernels.py \
    tests/test_gpu_model.py tests/test_gpu_train.py tests/test_gpu_aggregator.py tests/test_gpu_kernels.py -x -v -s --timeout 500 \
    --timeout-method thread || exit $?
fi
if [ "$WHAT" = benches ] || [ "$WHAT" = all ]; then
  step headline 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  step headline_attn16 240 env VGGT_ATTN16=1 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  step c3 300 python -u bench.py --config 3 --steps 3 --warmup 2 || exit $?
  step c3_eager_align 300 env VGGT_ALIGN_GRAPH=0 VGGT_ALIGN_PREFIX=0 python -u bench.py --config 3 --steps 3 --warmup 2 || exit $?
  step c2 300 python -u bench.py --config 2 --steps 3 --warmup 2 || exit $?
  step c0 240 python -u bench.py --config 0 --steps 10 --warmup 3 --no-cpu-baseline || exit $?
  step chunk 240 python -u bench.py --workload chunk --steps 5 --warmup 2 || exit $?
fi
echo "[$(date +%T)] done"
