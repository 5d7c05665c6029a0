#!/bin/bash
# Round-2 re-entry check: GPU parity suite, headline bench, GEMM shapes vs hipBLASLt
# and the hipBLASLt kernel names (kernel trace).  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit $?
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log"
timeout -k 10 300 python scripts/gemmbench.py --modes -1,9 --shapes fc2,proj,fc1 --epis torch,plain,resid > "$OUT/gemmbench.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/hbl -o run -- python3 scripts/hipblaslt_ref.py > "$OUT/hbl.log" 2>&1 || exit $?
python3 scripts/prof_summary.py /tmp/hbl/run_results.db > "$OUT/hbl_kernels.md" || exit $?
cat "$OUT/gemmbench.log" | grep -v '^{'
