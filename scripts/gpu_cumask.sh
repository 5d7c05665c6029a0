#!/bin/bash
# CU-mask placement probe, then the recurrence probe with the non-persistent GEMM forms
OUT=gpurun_out/${1:-cumask}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/probes/cumask_probe > "$OUT/probe.txt" 2>&1 || exit $?
cat "$OUT/probe.txt"
timeout -k 10 300 env VGGT_ALIGN_GRAPH=0 VGGT_GEMM_PERSIST=0 VGGT_PROBE_RESERVE=8 python -u bench.py --config 3 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/c3_nopersist.out" 2> "$OUT/c3_nopersist.err" || exit $?
echo done
