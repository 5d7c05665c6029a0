#!/bin/bash
# A/B of two builds of the library on the 154x518 sequence (configs[3]):
# lib/libvggt_old.so vs lib/libvggt_mi355x.so, alternating, after the GEMM tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${1:-ab_seq}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "gemm" > "$OUT/pytest_gemm.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_gemm.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for L in old mi355x; do
  VGGT_MI355X_LIB=$PWD/large-scale-vit-slam_amd/lib/libvggt_$L.so timeout -k 10 300 python bench.py --workload sequence --seq-frames 512 --height 154 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/seq_${L}_$r.log" 2>&1 || exit $?
  echo "$L $r $(tail -1 "$OUT/seq_${L}_$r.log" | cut -c1-160)"
done
done
