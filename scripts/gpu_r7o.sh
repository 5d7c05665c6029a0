#!/bin/bash
# DMA-placement bitwise test; tile-group height 16 vs 4 (and 32) again, aggregator + configs[3].  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "dma_placements" > "$OUT/pytest_pl.log" 2>&1 || { tail -20 "$OUT/pytest_pl.log"; exit 1; }
tail -1 "$OUT/pytest_pl.log"
run() {  # name, bench args (quoted), env...
  local n=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py $args --no-cpu-baseline > "$OUT/$n.tmp" 2>> "$OUT/err.log" || exit $?
  cat "$OUT/$n.tmp" >> "$OUT/$n.json"
  echo "$n: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['value'])" "$OUT/$n.tmp")"
}
for r in 1 2; do
  run agg_gm4 "" VGGT_GEMM_GM=4
  run agg_gm16 "" VGGT_GEMM_GM=16
  run agg_gm32 "" VGGT_GEMM_GM=32
done
run c3_gm4 "--config 3 --steps 2 --warmup 1" VGGT_GEMM_GM=4
run c3_gm16 "--config 3 --steps 2 --warmup 1" VGGT_GEMM_GM=16
