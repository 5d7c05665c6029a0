#!/bin/bash
# GPU parity suite (one pytest process, per-test timeout) -> gpurun_out/TAG/.
#   usage: bash scripts/gpu_tests.sh TAG [pytest args...]   (default: tests -m gpu)
set -u
TAG=${1:-tests}
shift || true
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(tests -m gpu)
echo "[$(date +%T)] pytest ${ARGS[*]}"
timeout -k 10 1000 python -u -m pytest -x -q -rf --timeout 240 --timeout-method thread "${ARGS[@]}" \
  > "$OUT/pytest.log" 2>&1
rc=$?
echo "[$(date +%T)] pytest rc=$rc"
tail -n 30 "$OUT/pytest.log"
exit $rc
