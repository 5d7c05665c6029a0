#!/bin/bash
# Pipeline refactor check + kernel trace of the grouped configs[3] sequence.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 600 python bench.py --workload sequence --seq-frames 512 --height 154 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_seq_c4.log" 2>&1 || exit $?
tail -1 "$OUT/bench_seq_c4.log" > "$OUT/bench_seq_c4.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/pseq -o run -- python3 bench.py --workload sequence --seq-frames 512 --height 154 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_seq.log" 2>&1 || exit $?
python3 scripts/prof_summary.py /tmp/pseq/run_results.db > "$OUT/seq_c4_kernels.md" || exit $?
python3 scripts/prof_gaps.py /tmp/pseq/run_results.db --last-s 1.4 > "$OUT/gaps_seq_c4.txt" || exit $?
head -1 "$OUT/gaps_seq_c4.txt"; cut -c1-200 "$OUT/bench_seq_c4.json"
