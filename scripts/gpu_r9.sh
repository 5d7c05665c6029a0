#!/bin/bash
# Round 5 lease: selected GPU tests, the sequence bench (ring model costs), the headline
# (MFMA peak probe) and the counter passes whose files bench.py reports (with provenance).
#   usage: VGGT_GIT_HEAD=<sha> bash scripts/gpu_r9.sh TAG [tests|seq|head|pmc|all] [pytest -k expr]
set -u
TAG=${1:-r9}
WHAT=${2:-all}
KEXPR=${3:-}
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  tail -n 3 "$OUT/$name.out"
  return $rc
}
has() { [ "$WHAT" = all ] || [[ ",$WHAT," == *",$1,"* ]]; }
if has seq; then
  step c3 400 python -u bench.py --config 3 --steps 3 --warmup 2 --no-cpu-baseline || exit $?
  grep '^{' "$OUT/c3.out" | tail -1 > "$OUT/c3.json"
fi
if has c4; then
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
if has head; then
  step headline 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit $?
  grep '^{' "$OUT/headline.out" | tail -1 > "$OUT/headline.json"
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
fi

if has kbench; then
  step kbench_attn 300 python -u scripts/kbench.py --only attn --attn-waves 8,4 --attn-variants ${ATTN_VARIANTS:-33,289} --rounds 2 --warm-s 2 || exit $?
fi
if has tests; then
  step pytest 900 python -u -m pytest ${TESTS:-tests/test_gpu_pipeline.py tests/test_gpu_gate.py tests/test_gpu_ring.py tests/test_gpu_fullsize.py} \
    --maxfail=5 -v -s --timeout 400 --timeout-method thread ${KEXPR:+-k "$KEXPR"} || exit $?
fi
echo "[$(date +%T)] done"
