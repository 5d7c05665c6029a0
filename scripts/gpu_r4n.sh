#!/bin/bash
# Grouped chunk encode in ChunkPipeline: parity, then sequence A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash scripts/ab_combo.sh $1_c4 "VGGT_ENCODE_GROUP=1 VGGT_ENCODE_GROUP=3" 2 --workload sequence --seq-frames 512 --height 154 --steps 2 --warmup 1 || exit $?
bash scripts/ab_combo.sh $1_c3 "VGGT_ENCODE_GROUP=1 VGGT_ENCODE_GROUP=3" 1 --workload sequence --seq-frames 64 --steps 2 --warmup 1 || exit $?
