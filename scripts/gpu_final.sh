#!/bin/bash
# the round-end checks on one box: the whole GPU suite, smoke, the default bench line and configs[3]
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
T=${1:-final}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 720 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > "$OUT/pytest.out" 2>&1 || { tail -30 "$OUT/pytest.out"; exit 1; }
tail -1 "$OUT/pytest.out"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.out" 2>&1 || { tail "$OUT/smoke.out"; exit 1; }
tail -1 "$OUT/smoke.out"
timeout -k 10 300 python -u bench.py > "$OUT/bench.out" 2> "$OUT/bench.err" || exit 1
grep '^{' "$OUT/bench.out" | tail -1 | cut -c1-300
timeout -k 10 400 python -u bench.py --config 3 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/c3.out" 2> "$OUT/c3.err" || exit 1
grep '^{' "$OUT/c3.out" | tail -1 | cut -c1-200
timeout -k 10 300 python -u bench.py --config 0 --steps 10 --warmup 3 > "$OUT/c0.out" 2> "$OUT/c0.err" || exit 1
grep '^{' "$OUT/c0.out" | tail -1 | cut -c1-200
