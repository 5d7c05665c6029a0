#!/bin/bash
# Bench (aggregator, chunk, train) + kernel-trace tables, summarised on the box
# (the databases stay behind, so the merge-back stays small).  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
P=/tmp/prof_$1
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
timeout -k 10 600 python bench.py --workload chunk --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_chunk.log" 2>&1 || exit $?
tail -1 "$OUT/bench_chunk.log" > "$OUT/bench_chunk.json"
timeout -k 10 600 python bench.py --workload train --steps 5 --warmup 2 > "$OUT/bench_train.log" 2>&1 || exit $?
tail -1 "$OUT/bench_train.log" > "$OUT/bench_train.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $P/agg -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit $?
python3 scripts/prof_summary.py $P/agg/run_results.db > "$OUT/aggregator_kernels.md" || exit $?
cp $P/agg/run_kernel_stats.csv "$OUT/aggregator_kernel_stats.csv" 2>/dev/null || true
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $P/chunk -o run -- python3 bench.py --workload chunk --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/prof_chunk.log" 2>&1 || exit $?
python3 scripts/prof_summary.py $P/chunk/run_results.db > "$OUT/full_chunk_kernels.md" || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $P/seq -o run -- python3 bench.py --workload sequence --seq-frames 512 --height 154 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_seq.log" 2>&1 || exit $?
python3 scripts/prof_summary.py $P/seq/run_results.db > "$OUT/seq_c4_kernels.md" || exit $?
cat "$OUT/bench.json"
