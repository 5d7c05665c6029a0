#!/bin/bash
# one lease: the whole GPU suite (as the driver runs it), then one bounded CPU-baseline run
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
T=${1:-r8n}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 720 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > "$OUT/pytest.out" 2>&1 || { tail -30 "$OUT/pytest.out"; exit 1; }
tail -2 "$OUT/pytest.out"
bash scripts/gpu_cpubase.sh C2 16 1 460 || exit $?
echo all done
