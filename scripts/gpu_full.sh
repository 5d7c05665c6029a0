#!/bin/bash
# Full GPU session: parity tests -> bench -> kernel-trace profiles (aggregator
# and full chunk) -> PMC HBM-traffic passes (FETCH_SIZE, WRITE_SIZE separately).
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
#   usage: bash scripts/gpu_full.sh TAG
set -u
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1; shift; local t=$1; shift; echo "[$(date +%T)] $name ..."; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; tail -n 3 "$OUT/$name.log"; return $rc; }
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest 1200 python -m pytest tests -m gpu -q -rf; rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: pytest rc=$rc"; exit $rc; fi
fi
step bench 900 python bench.py --steps 5 --warmup 2 || exit $?
step bench_chunk 900 python bench.py --workload chunk --steps 5 --warmup 2 --no-cpu-baseline || exit $?
step bench_train 900 python bench.py --workload train --steps 5 --warmup 2 || exit $?
step prof 900 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit $?
step prof_chunk 900 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_chunk" -o run -- python3 bench.py --workload chunk --steps 2 --warmup 1 --no-cpu-baseline || exit $?
step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline || exit $?
step pmc_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline || exit $?
python3 scripts/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --kernel attn_fwd_kernel --grid 704512 --out "$OUT/attn_traffic.json" || true
echo done
