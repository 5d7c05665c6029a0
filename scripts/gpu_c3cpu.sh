#!/bin/bash
# BASELINE.md §3 row C3 (the 64-frame full FeatureAlignedVGGT sequence on the oracle, 16 threads) in the
# background of one lease, resumable across leases (scripts/cpu_baseline_c3.py: the state comes back in
# gpurun_out/c3cpu/state.pt; copy it to scratch/c3cpu/state.pt before the next lease), with light GPU work
# (one launch thread) in the foreground.
#   usage: [GPU_WORK=1] bash scripts/gpu_c3cpu.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/c3cpu
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -f scratch/c3cpu/state.pt ] && [ ! -f "$OUT/state.pt" ]; then cp scratch/c3cpu/state.pt "$OUT/state.pt"; fi
timeout -k 10 "${CPU_S:-1110}" python -u scripts/cpu_baseline_c3.py --threads 16 --state "$OUT/state.pt" \
  --out "$OUT/cpu_baseline_full.json" --max-seconds "${CPU_BUDGET:-1060}" --chunk-estimate 500 > "$OUT/c3.log" 2>&1 &
CPID=$!
if [ "${GPU_WORK:-1}" = 1 ]; then
  P=/tmp/prof_c3cpu
  echo "[$(date +%T)] trace headline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/agg -o run -- python3 bench.py --steps 5 --warmup 2 \
    --no-cpu-baseline > "$OUT/prof.log" 2>&1 && python3 scripts/prof_summary.py $P/agg/run_results.db \
    > "$OUT/aggregator_kernels.md" && grep '^{' "$OUT/prof.log" | tail -1 > "$OUT/bench_under_rocprof.json"
  echo "[$(date +%T)] configs[2]"
  timeout -k 10 400 python3 -u bench.py --config 2 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/c2.out" 2>&1 \
    && grep '^{' "$OUT/c2.out" | tail -1 > "$OUT/c2.json"
  echo "[$(date +%T)] chunk"
  timeout -k 10 300 python3 -u bench.py --workload chunk --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/chunk.out" 2>&1 \
    && grep '^{' "$OUT/chunk.out" | tail -1 > "$OUT/chunk.json"
fi
echo "[$(date +%T)] waiting for the CPU sequence"
wait $CPID
echo "[$(date +%T)] cpu rc=$?"
tail -8 "$OUT/c3.log"
