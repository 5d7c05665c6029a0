#!/bin/bash
# End-of-session snapshot: GPU parity suite + smoke, bench lines for every workload,
# kernel-trace tables (scripts/gpu_bench_prof.sh).  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -1 "$OUT/smoke.log"
if [ -n "${AB_ADAM:-}" ]; then bash scripts/ab_env.sh $1 VGGT_ADAMW_FUSED "0 1" 2 --workload train --steps 5 --warmup 2 || exit $?; fi
bash scripts/gpu_bench_prof.sh $1 || exit $?
timeout -k 10 600 python bench.py --workload sequence --seq-frames 64 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_seq_c3.log" 2>&1 || exit $?
tail -1 "$OUT/bench_seq_c3.log" > "$OUT/bench_seq_c3.json"
timeout -k 10 600 python bench.py --workload sequence --seq-frames 512 --height 154 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_seq_c4.log" 2>&1 || exit $?
tail -1 "$OUT/bench_seq_c4.log" > "$OUT/bench_seq_c4.json"
for f in bench bench_chunk bench_train bench_seq_c3 bench_seq_c4; do python3 -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['ms_per_step'])"; done
