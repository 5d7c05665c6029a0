#!/bin/bash
# Sequence workloads (BASELINE configs[2]/[3]) on one GPU: benches + a kernel
# trace of the 512-frame 154x518 sequence.  usage: bash scripts/gpu_seq.sh TAG
set -u
TAG=${1:-seq}
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1; shift; local t=$1; shift; echo "[$(date +%T)] $name ..."; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; tail -n 1 "$OUT/$name.log" | cut -c1-400; return $rc; }
step bench_seq_c3 600 python bench.py --workload sequence --seq-frames 64 --steps 2 --warmup 1 --no-cpu-baseline || exit $?
step bench_seq_c4 600 python bench.py --workload sequence --seq-frames 512 --height 154 --steps 2 --warmup 1 --no-cpu-baseline || exit $?
step prof_seq_c4 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_seq_c4" -o run -- python3 bench.py --workload sequence --seq-frames 512 --height 154 --steps 1 --warmup 1 --no-cpu-baseline || exit $?
echo done
