#!/bin/bash
# one lease: pipeline / ring / full-size tests, configs[3] with the short-workgroup ring
# encode stream, then a bounded CPU-baseline slice (C2 at os.cpu_count() threads)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
T=${1:-r8m}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_small_kernels.py tests/test_gpu_pipeline.py tests/test_gpu_ring.py tests/test_gpu_fullsize.py -x -v -s \
  --timeout 600 --timeout-method thread > "$OUT/pytest.out" 2>&1 || exit $?
tail -2 "$OUT/pytest.out"
timeout -k 10 300 python -u bench.py --config 3 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/c3.out" 2> "$OUT/c3.err" || exit $?
grep '^{' "$OUT/c3.out" | tail -1 | cut -c1-160
bash scripts/gpu_cpubase.sh C2 0 3 420 || exit $?
echo all done
