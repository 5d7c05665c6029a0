#!/bin/bash
# Round-3 snapshot: GPU suite + smoke, the default bench line, the rocprofv3 kernel-trace --stats summary of that
# same command, the step's counter MFMA utilisation, and every workload's bench line.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
bash scripts/gpu_tests.sh "$1" || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench_err.log" || exit $?
cat "$OUT/bench.json"
P=/tmp/prof_$1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $P/agg -o run -- python3 bench.py > "$OUT/prof_bench.json" 2> "$OUT/prof.log" || exit $?
S=$(find $P/agg -name "*kernel_stats.csv" | head -1)
[ -n "$S" ] && cp "$S" "$OUT/bench_kernel_stats.csv"
ls -R $P/agg | head -20 > "$OUT/prof_files.txt"
python3 scripts/prof_summary.py $(find $P/agg -name "*results.db" | head -1) > "$OUT/aggregator_kernels.md" || exit $?
head -12 "$OUT/aggregator_kernels.md"
bash scripts/gpu_step_pmc.sh "$1" || exit $?
for w in "chunk:--workload chunk --steps 5 --warmup 2" "train:--workload train --steps 8 --warmup 3" \
         "c2:--config 2 --steps 2 --warmup 1" "c3:--config 3 --steps 2 --warmup 1" "c4:--config 4 --steps 2 --warmup 1"; do
  n=${w%%:*}; a=${w#*:}
  timeout -k 10 400 python3 bench.py $a --no-cpu-baseline > "$OUT/bench_$n.json" 2>> "$OUT/bench_err.log" || exit $?
  echo "$n: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['value'])" "$OUT/bench_$n.json")"
done
