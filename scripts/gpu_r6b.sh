#!/bin/bash
# Kernel traces of the training step and of configs[3] (512 frames 154x518): per-kernel tables + gap analysis
# of the last step.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
P=/tmp/prof_$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/train -o run -- python3 bench.py --workload train --steps 3 --warmup 1 > "$OUT/prof_train.log" 2>&1 || exit $?
python3 scripts/prof_summary.py $P/train/run_results.db > "$OUT/train_kernels.md" || exit $?
python3 scripts/prof_gaps.py $P/train/run_results.db --last-s 0.079 --top 25 > "$OUT/gaps_train.txt" || exit $?
python3 scripts/prof_names.py $P/train/run_results.db --last-s 0.079 > "$OUT/train_last_step_counts.txt" || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/c3 -o run -- python3 bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_c3.log" 2>&1 || exit $?
python3 scripts/prof_summary.py $P/c3/run_results.db > "$OUT/c3_kernels.md" || exit $?
python3 scripts/prof_gaps.py $P/c3/run_results.db --last-s 1.3 --top 25 > "$OUT/gaps_c3.txt" || exit $?
python3 scripts/prof_names.py $P/c3/run_results.db --last-s 1.3 > "$OUT/c3_last_step_counts.txt" || exit $?
