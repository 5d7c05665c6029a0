#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
T=${1:-r8r}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gate.py tests/test_gpu_pipeline.py tests/test_gpu_ring.py -x -v -s --timeout 500 --timeout-method thread > "$OUT/pytest.out" 2>&1 || { tail -30 "$OUT/pytest.out"; exit 1; }
tail -1 "$OUT/pytest.out"
timeout -k 10 400 python -u bench.py --config 3 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/c3.out" 2> "$OUT/c3.err" || { tail -20 "$OUT/c3.err"; exit 1; }
grep '^{' "$OUT/c3.out" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['recurrence']))"
bash scripts/gpu_queue_trace.sh $T || exit $?
