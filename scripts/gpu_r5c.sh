#!/bin/bash
# r5c: 154x518 sequence parity test, DPT conv microbench, conv / upsample PMC anatomy + traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r5c
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1; shift; local t=$1; shift; echo "[$(date +%T)] $name ..."; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; tail -n 4 "$OUT/$name.log"; return $rc; }
step pytest 400 python -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -m gpu -s -k vkitti
step pytest_dpt 400 python -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_model.py -m gpu -k "heads or dpt or two_chunks or given_oracle" || exit $?
step dpt_ab 300 python scripts/dpt_ab.py --rounds 5 || exit $?
step convbench 200 python scripts/convbench_pre.py --reps 10 || exit $?
for k in c148 c518 up; do
  GRID= step pmc_$k 300 bash scripts/kernel_pmc.sh r5c/anat_$k "$( [ $k = up ] && echo upsample_kernel || echo conv_pre_kernel )" python3 scripts/convbench_pre.py --reps 2 --only $k || exit $?
  step fetch_$k 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$k -o run -- python3 scripts/convbench_pre.py --reps 2 --only $k || exit $?
  step write_$k 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_$k -o run -- python3 scripts/convbench_pre.py --reps 2 --only $k || exit $?
done
echo done
