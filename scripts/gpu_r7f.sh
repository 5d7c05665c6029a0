#!/bin/bash
# New defaults vs the r7b library on the other workloads: configs[3] sequence, full chunk, training.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
L=$PWD/large-scale-vit-slam_amd/lib
run() {  # name, bench args (quoted), env...
  local n=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py $args --no-cpu-baseline > "$OUT/$n.tmp" 2>> "$OUT/err.log" || exit $?
  cat "$OUT/$n.tmp" >> "$OUT/$n.json"
  echo "$n: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['value'])" "$OUT/$n.tmp")"
}
OLDENV="VGGT_MI355X_LIB=$L/libvggt_r7b.so VGGT_GEMM_PIPE=0 VGGT_ATTN16=0"
for r in 1 2; do
  run c3_old "--config 3 --steps 2 --warmup 1" $OLDENV
  run c3_new "--config 3 --steps 2 --warmup 1"
  run chunk_old "--workload chunk --steps 5 --warmup 2" $OLDENV
  run chunk_new "--workload chunk --steps 5 --warmup 2"
  run train_old "--workload train --steps 8 --warmup 3" $OLDENV
  run train_new "--workload train --steps 8 --warmup 3"
done
