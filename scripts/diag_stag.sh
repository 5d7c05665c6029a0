#!/bin/bash
# staggered attention: bitwise parity vs variant 33, then the A/B timing
OUT=gpurun_out/${1:-stag}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  -k "staggered_equals_lockstep or offset_free_extremes or eight_wave" > "$OUT/pytest.out" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.out"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/attn_stag_bench.py > "$OUT/ab.out" 2>&1
rc=$?; echo "ab rc=$rc"; cat "$OUT/ab.out"; exit $rc
