#!/bin/bash
# GEMM shapes vs hipBLASLt and the hipBLASLt kernel names (kernel trace).  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python scripts/gemmbench.py --modes=-1,9 --shapes fc2,proj,fc1 --epis torch,plain,resid > "$OUT/gemmbench.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/hbl -o run -- python3 scripts/hipblaslt_ref.py > "$OUT/hbl.log" 2>&1 || exit $?
python3 scripts/prof_summary.py /tmp/hbl/run_results.db > "$OUT/hbl_kernels.md" || exit $?
grep -v '^{' "$OUT/gemmbench.log"
