#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 600 python bench.py --workload sequence --seq-frames 64 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_seq_c3.log" 2>&1 || exit $?
tail -1 "$OUT/bench_seq_c3.log" | tee "$OUT/bench_seq_c3.json"
timeout -k 10 600 python bench.py --workload sequence --seq-frames 512 --height 154 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_seq_c4.log" 2>&1 || exit $?
tail -1 "$OUT/bench_seq_c4.log" | tee "$OUT/bench_seq_c4.json"
