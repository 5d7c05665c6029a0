#!/bin/bash
# Final check of the committed tree: GPU suite, smoke, default bench line.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
bash scripts/gpu_tests.sh "$1" || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench_err.log" || exit $?
cat "$OUT/bench.json"
