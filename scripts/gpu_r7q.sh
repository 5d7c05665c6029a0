#!/bin/bash
# Kernel tables of the full per-chunk FeatureAlignedVGGT and the training step with the round-3 defaults.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
P=/tmp/prof_$1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $P/chunk -o run -- python3 bench.py --workload chunk --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/prof_chunk.json" 2> "$OUT/prof_chunk.log" || exit $?
python3 scripts/prof_summary.py $(find $P/chunk -name "*results.db" | head -1) > "$OUT/full_chunk_kernels.md" || exit $?
head -24 "$OUT/full_chunk_kernels.md"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $P/train -o run -- python3 bench.py --workload train --steps 4 --warmup 2 --no-cpu-baseline > "$OUT/prof_train.json" 2> "$OUT/prof_train.log" || exit $?
python3 scripts/prof_summary.py $(find $P/train -name "*results.db" | head -1) > "$OUT/train_kernels.md" || exit $?
head -16 "$OUT/train_kernels.md"
