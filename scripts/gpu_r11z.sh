#!/bin/bash
# Round 6, final tree: the whole GPU suite, smoke, the default bench line (with its CPU baseline), its
# rocprofv3 kernel-trace summary, the counter passes bench.py reports (HBM traffic of the global attention,
# MFMA utilisation of the step; stamped with the source fingerprint), and the other BASELINE configs.
#   usage: VGGT_GIT_HEAD=<sha> bash scripts/gpu_r11z.sh TAG [tests,smoke,head,prof,pmc,seq,c2,chunk,c0 | all]
set -u
TAG=${1:-r11z}
WHAT=${2:-all}
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
has() { [ "$WHAT" = all ] || [[ ",$WHAT," == *",$1,"* ]]; }
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  tail -n 2 "$OUT/$name.out" | cut -c1-400
  return $rc
}
if has tests; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread || exit $?
fi
if has smoke; then
  step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if has head; then
  step headline 400 python -u bench.py || exit $?
  grep '^{' "$OUT/headline.out" | tail -1 > "$OUT/headline.json"
fi
if has prof; then
  echo "[$(date +%T)] rocprof kernel trace"
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 \
    --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit $?
  DB=$(find /tmp/prof_$TAG -name '*.db' | head -1)
  python3 scripts/prof_summary.py "$DB" > "$OUT/aggregator_kernels.md" || exit $?
  find /tmp/prof_$TAG -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
  head -8 "$OUT/aggregator_kernels.md"
fi
if has pmc; then
  P=/tmp/pmc_$TAG
  CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
  export VGGT_MFMA_PROBE=0
  echo "[$(date +%T)] pmc fetch"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/f -o run -- $CMD > "$OUT/pmc_f.log" 2>&1 || exit $?
  echo "[$(date +%T)] pmc write"
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/w -o run -- $CMD > "$OUT/pmc_w.log" 2>&1 || exit $?
  python3 scripts/pmc_traffic.py $P/f $P/w --kernel attn_fwd_kernel --grid 704512 --out "$OUT/attn_traffic.json" || exit $?
  echo "[$(date +%T)] pmc step"
  BENCH="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline"
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $P/busy -o run -- $BENCH > "$OUT/busy.log" 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE --output-format csv -d $P/mops -o run -- $BENCH > "$OUT/mops.log" 2>&1 || exit $?
  python3 scripts/step_pmc.py $P/busy $P/mops --out "$OUT/step_mfma.json" || exit $?
  unset VGGT_MFMA_PROBE
fi
if has seq; then
  step c3 400 python -u bench.py --config 3 --steps 3 --warmup 2 --no-cpu-baseline || exit $?
  grep '^{' "$OUT/c3.out" | tail -1 > "$OUT/c3.json"
  step c4 400 python -u bench.py --config 4 --steps 3 --warmup 2 --no-cpu-baseline || exit $?
  grep '^{' "$OUT/c4.out" | tail -1 > "$OUT/c4.json"
fi
if has c2; then
  step c2 400 python -u bench.py --config 2 --steps 2 --warmup 1 || exit $?
  grep '^{' "$OUT/c2.out" | tail -1 > "$OUT/c2.json"
fi
if has chunk; then
  step chunk 300 python -u bench.py --workload chunk --steps 10 --warmup 3 --no-cpu-baseline || exit $?
  grep '^{' "$OUT/chunk.out" | tail -1 > "$OUT/chunk.json"
fi
if has c0; then
  step c0 300 python -u bench.py --config 0 --steps 10 --warmup 3 || exit $?
  grep '^{' "$OUT/c0.out" | tail -1 > "$OUT/c0.json"
fi
echo "[$(date +%T)] done"
