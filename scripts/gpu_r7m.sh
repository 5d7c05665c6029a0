#!/bin/bash
# GEMM DMA placement 64 (half 1 issues its W pieces after the MFMAs of MATH(j) for K-tile j+2; every READ segment
# at most 8 pieces) against the default 5: GEMM tests, bitwise + timings, aggregator and configs[3].  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
VGGT_GEMM_PIPE=64 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "gemm" > "$OUT/pytest_p64.log" 2>&1 || { tail -20 "$OUT/pytest_p64.log"; exit 1; }
tail -1 "$OUT/pytest_p64.log"
timeout -k 10 240 python3 -u scripts/pipebench.py --pipes 5,64 > "$OUT/pipebench.txt" 2>&1 || { tail -5 "$OUT/pipebench.txt"; exit 1; }
grep -v bitwise "$OUT/pipebench.txt"
run() {  # name, bench args (quoted), env...
  local n=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py $args --no-cpu-baseline > "$OUT/$n.tmp" 2>> "$OUT/err.log" || exit $?
  cat "$OUT/$n.tmp" >> "$OUT/$n.json"
  echo "$n: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['value'])" "$OUT/$n.tmp")"
}
for r in 1 2; do
  run agg_p5 ""
  run agg_p64 "" VGGT_GEMM_PIPE=64
done
run c3_p5 "--config 3 --steps 2 --warmup 1"
run c3_p64 "--config 3 --steps 2 --warmup 1" VGGT_GEMM_PIPE=64
