#!/bin/bash
# Host-side pose algebra for no-grad inference: parity, then sequence / chunk A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_align.py tests/test_gpu_train.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash scripts/ab_env.sh $1_c4 VGGT_HOST_POSE "0 1" 2 --workload sequence --seq-frames 512 --height 154 --steps 2 --warmup 1 || exit $?
bash scripts/ab_env.sh $1_chunk VGGT_HOST_POSE "0 1" 2 --workload chunk --steps 4 --warmup 2 || exit $?
