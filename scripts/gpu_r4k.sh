#!/bin/bash
# wgrad by LDS-DMA: parity, kernel A/B, training A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for r in 1 2; do for p in 0 1; do VGGT_WGRAD_DMA=$p timeout -k 10 200 python scripts/wgrad_probe.py 2>&1 | grep dma= ; done; done
bash scripts/ab_env.sh $1 VGGT_WGRAD_DMA "0 1" 2 --workload train --steps 5 --warmup 2
