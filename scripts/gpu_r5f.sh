#!/bin/bash
# r5f: fused upsample+conv parity + bench, DPT A/B, full chunk
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r5f
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1; shift; local t=$1; shift; echo "[$(date +%T)] $name ..."; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; tail -n 3 "$OUT/$name.log"; return $rc; }
step pytest 500 python -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_small_kernels.py tests/test_gpu_model.py -m gpu -k "upsample or heads or dpt or two_chunks or given_oracle" || exit $?
step convbench 200 python scripts/convbench_pre.py --reps 10 --only fused || exit $?
step convbench_c518 200 python scripts/convbench_pre.py --reps 10 --only c518 || exit $?
step dpt_ab 300 python scripts/dpt_ab.py --rounds 5 || exit $?
step chunk 300 python bench.py --workload chunk --steps 5 --warmup 2 --no-cpu-baseline || exit $?
echo done
