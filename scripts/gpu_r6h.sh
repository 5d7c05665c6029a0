#!/bin/bash
# HIP_FORCE_DEV_KERNARG A/B (kernel arguments in device memory) on the aggregator step, the training step and
# configs[3].  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
for m in 0 1 0 1; do
  HIP_FORCE_DEV_KERNARG=$m timeout -k 10 200 python3 bench.py --no-cpu-baseline >> "$OUT/agg_$m.json" 2>> "$OUT/err.log" || exit $?
  HIP_FORCE_DEV_KERNARG=$m timeout -k 10 200 python3 bench.py --workload train --steps 10 --warmup 3 >> "$OUT/train_$m.json" 2>> "$OUT/err.log" || exit $?
done
for m in 0 1; do
  HIP_FORCE_DEV_KERNARG=$m timeout -k 10 300 python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline >> "$OUT/c3_$m.json" 2>> "$OUT/err.log" || exit $?
done
for f in "$OUT"/*.json; do echo "$f"; python3 -c "import json,sys; [print(' ', json.loads(l)['ms_per_step']) for l in open(sys.argv[1])]" "$f"; done
