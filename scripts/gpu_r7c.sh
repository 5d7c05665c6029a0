#!/bin/bash
# GEMM DMA placement (pipe 1 / 5), whole-K qkv, vectorised bf16 packing: GEMM tests under the variants, kernel
# timings, aggregator A/B against the r7b library.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
VGGT_GEMM_PIPE=5 VGGT_GEMM_FULLK=7 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "gemm" > "$OUT/pytest_gemm_p5.log" 2>&1 || { tail -20 "$OUT/pytest_gemm_p5.log"; exit 1; }
tail -1 "$OUT/pytest_gemm_p5.log"
timeout -k 10 240 python3 -u scripts/pipebench.py --pipes 0,1,5 > "$OUT/pipebench.txt" 2>&1 || { tail -5 "$OUT/pipebench.txt"; exit 1; }
grep -v bitwise "$OUT/pipebench.txt"
OLD=$PWD/large-scale-vit-slam_amd/lib/libvggt_r7b.so
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu-baseline > "$OUT/$n.tmp" 2>> "$OUT/err.log" || exit $?
  cat "$OUT/$n.tmp" >> "$OUT/$n.json"
  echo "$n: $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" "$OUT/$n.tmp")"
}
for r in 1 2; do
  run old VGGT_MI355X_LIB=$OLD VGGT_GEMM_PIPE=0 VGGT_ATTN16=0
  run p1 VGGT_GEMM_PIPE=1 VGGT_ATTN16=2
  run p5 VGGT_GEMM_PIPE=5 VGGT_ATTN16=2
  run p5fk VGGT_GEMM_PIPE=5 VGGT_ATTN16=2 VGGT_GEMM_FULLK=7
done
