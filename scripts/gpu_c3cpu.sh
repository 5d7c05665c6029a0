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
  VGGT_MFMA_PROBE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/agg -o run -- python3 bench.py --steps 5 \
    --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1 && python3 scripts/prof_summary.py $P/agg/run_results.db \
    > "$OUT/aggregator_kernels.md" && grep '^{' "$OUT/prof.log" | tail -1 > "$OUT/bench_under_rocprof.json"
  echo "[$(date +%T)] train"
  timeout -k 10 300 python3 -u bench.py --workload train --steps 10 --warmup 3 > "$OUT/train.out" 2>&1 \
    && grep '^{' "$OUT/train.out" | tail -1 > "$OUT/train.json"
  echo "[$(date +%T)] attention anatomy"
  CMD="python3 scripts/kbench.py --only attn --attn-waves 8 --attn-variants 33 --reps 8 --warm-s 1"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $P/p1 -o run -- $CMD > "$OUT/anat1.log" 2>&1 \
    && timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS --output-format csv -d $P/p2 -o run -- $CMD > "$OUT/anat2.log" 2>&1 \
    && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $P/p3 -o run -- $CMD > "$OUT/anat3.log" 2>&1 \
    && python3 scripts/pmc_anatomy.py $P/p1 $P/p2 $P/p3 --kernel attn_fwd_kernel > "$OUT/attn_anatomy.md" 2>&1
fi
echo "[$(date +%T)] waiting for the CPU sequence"
wait $CPID
echo "[$(date +%T)] cpu rc=$?"
tail -8 "$OUT/c3.log"
