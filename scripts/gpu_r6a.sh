#!/bin/bash
# Round-3 late check: full GPU suite, smoke, default bench, training-step graph A/B, step PMC.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r6a
mkdir -p "$OUT"
export TMPDIR=/tmp
bash scripts/gpu_tests.sh r6a || exit $?
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
echo "[$(date +%T)] smoke ok"
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
cat "$OUT/bench.json"
for gmode in 0 1 0 1; do
  VGGT_TRAIN_GRAPH=$gmode timeout -k 10 200 python3 bench.py --workload train --steps 10 --warmup 3 \
    >> "$OUT/train_ab.json" 2>> "$OUT/train_ab.err" || exit $?
done
cat "$OUT/train_ab.json"
bash scripts/gpu_step_pmc.sh r6a
