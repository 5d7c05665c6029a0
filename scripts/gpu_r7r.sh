#!/bin/bash
# The GELU + pre-activation GEMM of the training step on the whole-K-tile loop (VGGT_GEMM_FULLK=13) vs 5.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
VGGT_GEMM_FULLK=13 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "gelu_pre or gemm_production" > "$OUT/pytest_fk13.log" 2>&1 || { tail -20 "$OUT/pytest_fk13.log"; exit 1; }
tail -1 "$OUT/pytest_fk13.log"
for r in 1 2; do
  for f in 5 13; do
    VGGT_GEMM_FULLK=$f timeout -k 10 300 python3 bench.py --workload train --steps 8 --warmup 3 --no-cpu-baseline > "$OUT/fk$f.tmp" 2>> "$OUT/err.log" || exit $?
    cat "$OUT/fk$f.tmp" >> "$OUT/fk$f.json"
    echo "fullk $f: $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" "$OUT/fk$f.tmp")"
  done
done
