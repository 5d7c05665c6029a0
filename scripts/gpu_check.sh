#!/bin/bash
# One GPU-box session: GPU parity tests -> bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script
# (pytest exit 1 = ordinary test failures, which do not stop later steps).
#   usage: bash scripts/gpu_check.sh TAG [pytest-args...]
set -u
TAG=${1:-run}; shift || true
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1; shift; local t=$1; shift; echo "[$(date +%T)] $name ..."; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; tail -n 5 "$OUT/$name.log"; return $rc; }
step pytest 1200 python -m pytest tests -m gpu -q -rf "$@"; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: pytest rc=$rc"; exit $rc; fi
[ -n "${SKIP_BENCH:-}" ] && { echo "bench skipped"; exit 0; }
step bench 900 python bench.py --steps 5 --warmup 2 || exit $?
step prof 900 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof" -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit $?
echo done
