#!/bin/bash
# r5e: host syncs per chunk, pose-kernel A/B on configs[3]/[4] + full chunk, headline bench, step PMC
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r5e
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1; shift; local t=$1; shift; echo "[$(date +%T)] $name ..."; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; tail -n 2 "$OUT/$name.log"; return $rc; }
step sync_probe 300 python scripts/sync_probe.py || exit $?
for r in 1 2; do
  for mode in host hip; do
    step c3_${mode}_$r 300 env VGGT_POSE=$mode python bench.py --config 3 --steps 3 --warmup 1 || exit $?
    step chunk_${mode}_$r 300 env VGGT_POSE=$mode python bench.py --workload chunk --steps 5 --warmup 2 --no-cpu-baseline || exit $?
  done
done
step c4 300 python bench.py --config 4 --steps 3 --warmup 1 || exit $?
step c2 300 python bench.py --config 2 --steps 3 --warmup 1 || exit $?
step bench 600 python bench.py --steps 10 --warmup 3 || exit $?
step mops_cal 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE --output-format csv -d $OUT/mops_cal -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline || exit $?
echo done
