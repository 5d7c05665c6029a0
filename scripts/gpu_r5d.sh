#!/bin/bash
# r5d: DPT A/B (reorder + separable pos), parity tests touched, in-model GEMM anatomy, step MFMA counters
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r5d
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1; shift; local t=$1; shift; echo "[$(date +%T)] $name ..."; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; tail -n 4 "$OUT/$name.log"; return $rc; }
step pytest 500 python -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_small_kernels.py tests/test_gpu_model.py -m gpu -s -k "vkitti or separable or heads or dpt or two_chunks" || exit $?
step dpt_ab 300 python scripts/dpt_ab.py --rounds 5 || exit $?
step stepmfma 600 bash scripts/gpu_step_pmc.sh r5d || exit $?
GRID= step anat_fc1 300 bash scripts/kernel_pmc.sh r5d/anat_fc1 "gemm_ppp_kernel<1," python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline || exit $?
GRID= step anat_qkv 300 bash scripts/kernel_pmc.sh r5d/anat_qkv "gemm_ppp_kernel<16," python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline || exit $?
GRID= step anat_attn 300 bash scripts/kernel_pmc.sh r5d/anat_attn "attn_fwd_kernel<64, 8" python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline || exit $?
echo done
