#!/bin/bash
# Knockout timing of the persistent GEMM (diagnostic builds, wrong results): no in-loop DMA, no epilogue math,
# both -- against the default library.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
L=$PWD/large-scale-vit-slam_amd/lib
for r in 1 2; do
for v in mi355x ko_dma ko_epi ko_both; do
  VGGT_MI355X_LIB=$L/libvggt_$v.so timeout -k 10 200 python3 -u scripts/pipebench.py --pipes 5 --rounds 2 > "$OUT/pb_$v.txt" 2>&1 || exit 1
  grep -v bitwise "$OUT/pb_$v.txt" | grep -v amdgpu.ids | sed "s/^/$v /"
done
done
