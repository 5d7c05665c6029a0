#!/bin/bash
# kernel trace of the overlapped configs[3] schedule (W = 1 ring with the default gated encode): per-queue busy / gaps
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
T=${1:-queue_trace}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
P=/tmp/prof_$T
timeout -k 10 400 env VGGT_OVERLAP_ALIGN=1 VGGT_RECURRENCE_PROBE=0 rocprofv3 --kernel-trace --output-format csv -d $P/ov -o run -- python3 bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || exit $?
python3 scripts/queue_gaps.py $P/ov > "$OUT/queues.txt" || exit $?
cat "$OUT/queues.txt"
