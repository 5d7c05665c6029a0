#!/bin/bash
# FK loop specialised for the default DMA placement: full GPU suite, aggregator and configs[3] A/B against
# the r7g library.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
L=$PWD/large-scale-vit-slam_amd/lib
bash scripts/gpu_tests.sh "$1" || exit $?
VGGT_GEMM_PIPE=37 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "gemm" > "$OUT/pytest_gemm_p37.log" 2>&1 || { tail -20 "$OUT/pytest_gemm_p37.log"; exit 1; }
tail -1 "$OUT/pytest_gemm_p37.log"
timeout -k 10 240 python3 -u scripts/pipebench.py --pipes 5,37 > "$OUT/pipebench.txt" 2>&1 || { tail -5 "$OUT/pipebench.txt"; exit 1; }
grep -v bitwise "$OUT/pipebench.txt"
run() {  # name, bench args (quoted), env...
  local n=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py $args --no-cpu-baseline > "$OUT/$n.tmp" 2>> "$OUT/err.log" || exit $?
  cat "$OUT/$n.tmp" >> "$OUT/$n.json"
  echo "$n: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['value'])" "$OUT/$n.tmp")"
}
for r in 1 2; do
  run agg_r7g "" VGGT_MI355X_LIB=$L/libvggt_r7g.so
  run agg_new ""
  run agg_p37 "" VGGT_GEMM_PIPE=37
done
run c3_r7g "--config 3 --steps 2 --warmup 1" VGGT_MI355X_LIB=$L/libvggt_r7g.so
run c3_new "--config 3 --steps 2 --warmup 1"
