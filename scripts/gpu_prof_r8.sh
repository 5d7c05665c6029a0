#!/bin/bash
# Round-4 evidence: kernel-trace tables of the headline and of the full chunk, and the
# DPT-conv HBM traffic (FETCH_SIZE / WRITE_SIZE passes + a trace pass, pmc_kernel_table.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
P=/tmp/prof_$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/agg -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit $?
grep '^{' "$OUT/prof.log" | tail -1 > "$OUT/bench_under_rocprof.json"
python3 scripts/prof_summary.py $P/agg/run_results.db > "$OUT/aggregator_kernels.md" || exit $?
cp $P/agg/run_kernel_stats.csv "$OUT/aggregator_kernel_stats.csv" 2>/dev/null || true
echo "headline traced"
CMD="python3 bench.py --workload chunk --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/f -o run -- $CMD > "$OUT/pmc_f.log" 2>&1 || exit $?
echo "fetch pass"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/w -o run -- $CMD > "$OUT/pmc_w.log" 2>&1 || exit $?
echo "write pass"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/t -o run -- $CMD > "$OUT/trace_chunk.log" 2>&1 || exit $?
python3 scripts/pmc_kernel_table.py $P/f $P/w $P/t --match conv,upsample,dpt --out "$OUT/dpt_traffic.md" || exit $?
python3 scripts/pmc_kernel_table.py $P/f $P/w $P/t --out "$OUT/chunk_traffic_all.md" > /dev/null || exit $?
cat "$OUT/dpt_traffic.md"
