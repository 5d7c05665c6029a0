#!/bin/bash
# recurrence probe: configs[3] sequence with graph-replayed vs eager alignment
OUT=gpurun_out/${1:-rec}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config 3 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/c3.out" 2> "$OUT/c3.err" || exit $?
tail -1 "$OUT/c3.out" | cut -c1-200
timeout -k 10 300 env VGGT_ALIGN_GRAPH=0 python -u bench.py --config 3 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/c3_eager.out" 2> "$OUT/c3_eager.err" || exit $?
echo done
