#!/bin/bash
# Gradient arena (one zero fill per backward): training parity, then A/B on the training bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash scripts/ab_env.sh $1 VGGT_GRAD_ARENA "0 1" 3 --workload train --steps 5 --warmup 2
