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
run() {  # name, bench args (quoted), env...
  local n=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py $args --no-cpu-baseline > "$OUT/$n.tmp" 2>> "$OUT/err.log" || exit $?
  cat "$OUT/$n.tmp" >> "$OUT/$n.json"
  echo "$n: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['value'])" "$OUT/$n.tmp")"
}
for r in 1 2; do
  run agg_r7g "" VGGT_MI355X_LIB=$L/libvggt_r7g.so
  run agg_new ""
done
run c3_r7g "--config 3 --steps 2 --warmup 1" VGGT_MI355X_LIB=$L/libvggt_r7g.so
run c3_new "--config 3 --steps 2 --warmup 1"
