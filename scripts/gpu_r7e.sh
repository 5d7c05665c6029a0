#!/bin/bash
# Branch-free grouped GELU lookups + whole-K-only DMA placement: GEMM tests, kernel timings against the r7d
# library, aggregator A/B, and a kernel trace of the new default.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
L=$PWD/large-scale-vit-slam_amd/lib
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "gemm" > "$OUT/pytest_gemm.log" 2>&1 || { tail -20 "$OUT/pytest_gemm.log"; exit 1; }
tail -1 "$OUT/pytest_gemm.log"
VGGT_MI355X_LIB=$L/libvggt_r7d.so timeout -k 10 240 python3 -u scripts/pipebench.py --pipes 5 > "$OUT/pipebench_r7d.txt" 2>&1 || exit 1
timeout -k 10 240 python3 -u scripts/pipebench.py --pipes 5 > "$OUT/pipebench_new.txt" 2>&1 || exit 1
grep -v bitwise "$OUT/pipebench_r7d.txt" | sed 's/^/r7d /'
grep -v bitwise "$OUT/pipebench_new.txt" | sed 's/^/new /'
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu-baseline > "$OUT/$n.tmp" 2>> "$OUT/err.log" || exit $?
  cat "$OUT/$n.tmp" >> "$OUT/$n.json"
  echo "$n: $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" "$OUT/$n.tmp")"
}
for r in 1 2; do
  run old VGGT_MI355X_LIB=$L/libvggt_r7b.so VGGT_GEMM_PIPE=0 VGGT_ATTN16=0
  run r7d VGGT_MI355X_LIB=$L/libvggt_r7d.so VGGT_GEMM_PIPE=5
  run new
  run new_bm192 VGGT_GEMM_BM=192
done
P=/tmp/prof_$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/agg -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit $?
python3 scripts/prof_summary.py $P/agg/run_results.db > "$OUT/aggregator_kernels.md" || exit $?
head -14 "$OUT/aggregator_kernels.md"
