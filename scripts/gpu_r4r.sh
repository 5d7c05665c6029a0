#!/bin/bash
# Grouped encode at 518^2 (two chunks per encode, DPT head per chunk): parity of the split DPT path, configs[2] A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash scripts/ab_combo.sh $1_c3 "VGGT_GROUP_TOKENS=24576 VGGT_GROUP_TOKENS=49152" 2 --workload sequence --seq-frames 64 --steps 2 --warmup 1 || exit $?
