#!/bin/bash
# 16x16x32 global attention as default: full GPU suite, bench A/B (VGGT_ATTN16 0/1 alternating), kernel-trace
# stats, HBM traffic PMC of the new kernel, step MFMA counters.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
bash scripts/gpu_tests.sh "$1" || exit $?
for m in 0 1 0 1; do
  VGGT_ATTN16=$m timeout -k 10 300 python3 bench.py --no-cpu-baseline >> "$OUT/bench_ab.json" 2>> "$OUT/bench_ab.err" || exit $?
done
cut -c1-200 "$OUT/bench_ab.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p6d/agg -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit $?
python3 scripts/prof_summary.py /tmp/p6d/agg/run_results.db > "$OUT/aggregator_kernels.md" || exit $?
cp /tmp/p6d/agg/run_kernel_stats.csv "$OUT/aggregator_kernel_stats.csv" 2>/dev/null || true
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/p6d/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/p6d/pmc_write -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1 || exit $?
python3 scripts/pmc_traffic.py /tmp/p6d/pmc_fetch /tmp/p6d/pmc_write --kernel attn16_fwd_kernel --grid 704512 --out "$OUT/attn_traffic.json" || exit $?
bash scripts/gpu_step_pmc.sh "$1"
for m in 0 1; do
  VGGT_ATTN16=$m timeout -k 10 300 python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline >> "$OUT/bench_c3_ab.json" 2>> "$OUT/bench_c3_ab.err" || exit $?
done
cut -c1-200 "$OUT/bench_c3_ab.json"
