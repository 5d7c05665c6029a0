#!/bin/bash
# Training-path launch cuts: training tests, training bench x3, last-step launch anatomy.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --workload train --steps 10 --warmup 3 >> "$OUT/train.json" 2>> "$OUT/train.err" || exit $?
done
cut -c1-230 "$OUT/train.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p6g/train -o run -- python3 bench.py --workload train --steps 3 --warmup 1 > "$OUT/prof_train.log" 2>&1 || exit $?
python3 scripts/prof_gaps.py /tmp/p6g/train/run_results.db --last-s 0.079 --top 10 > "$OUT/gaps_train.txt" || exit $?
python3 scripts/prof_names.py /tmp/p6g/train/run_results.db --last-s 0.079 > "$OUT/train_last_step_counts.txt" || exit $?
head -1 "$OUT/gaps_train.txt"; head -1 "$OUT/train_last_step_counts.txt"
