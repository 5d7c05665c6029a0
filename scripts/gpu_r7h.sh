#!/bin/bash
# FK loop specialised for the default DMA placement; bias values loaded before the next tile's DMA
# (diagnostic, VGGT_EPI_BIAS_EARLY); epilogue knockout -- GEMM tests + timings.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
L=$PWD/large-scale-vit-slam_amd/lib
for v in mi355x epi_bias_early; do
  VGGT_MI355X_LIB=$L/libvggt_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_kernels.py -k "gemm" > "$OUT/pytest_$v.log" 2>&1 || { tail -20 "$OUT/pytest_$v.log"; exit 1; }
  echo "$v $(tail -1 $OUT/pytest_$v.log)"
done
for r in 1 2; do
for v in r7g mi355x epi_bias_early ko_epi; do
  VGGT_MI355X_LIB=$L/libvggt_$v.so timeout -k 10 200 python3 -u scripts/pipebench.py --pipes 5 --rounds 2 > "$OUT/pb_$v.txt" 2>&1 || exit 1
  grep -v bitwise "$OUT/pb_$v.txt" | grep -v amdgpu.ids | sed "s/^/$v /"
done
done
