#!/bin/bash
# DPT conv (pre-split form): this K-step's fragment reads before the next step's DMA issue (-DVGGT_CONV_STAGE_LATE)
# against the default: conv tests, convbench, full chunk.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
L=$PWD/large-scale-vit-slam_amd/lib
VGGT_MI355X_LIB=$L/libvggt_convlate.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_small_kernels.py -k "conv" > "$OUT/pytest_convlate.log" 2>&1 || { tail -20 "$OUT/pytest_convlate.log"; exit 1; }
tail -1 "$OUT/pytest_convlate.log"
for r in 1 2; do
  for v in mi355x convlate; do
    VGGT_MI355X_LIB=$L/libvggt_$v.so timeout -k 10 200 python3 -u scripts/convbench_pre.py --reps 10 > "$OUT/cb_$v.txt" 2>&1 || exit 1
    grep -v amdgpu.ids "$OUT/cb_$v.txt" | sed "s/^/$v /"
  done
done
for r in 1 2; do
  for v in mi355x convlate; do
    VGGT_MI355X_LIB=$L/libvggt_$v.so timeout -k 10 300 python3 bench.py --workload chunk --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/chunk_$v.tmp" 2>> "$OUT/err.log" || exit $?
    cat "$OUT/chunk_$v.tmp" >> "$OUT/chunk_$v.json"
    echo "chunk $v: $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" "$OUT/chunk_$v.tmp")"
  done
done
