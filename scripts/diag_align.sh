#!/bin/bash
# Alignment-path parity under the three align modes (eager whole head / eager with
# the encode-side prefix / graph-replayed recurrence).  A step that ends other than
# pass (0) or test failure (1) stops the script.
OUT=gpurun_out/${1:-diag}
mkdir -p "$OUT"
export TMPDIR=/tmp
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
K="given_oracle_tokens or alignment_head_bf16"
run() {  # run NAME ENV...
  local name=$1; shift
  timeout -k 10 300 env "$@" $T tests/test_gpu_model.py -k "$K" > "$OUT/$name.out" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -E "^chunk|^sim3|passed|failed" "$OUT/$name.out" | tail -6
  [ $rc -le 1 ]
}
timeout -k 10 400 $T tests/test_gpu_kernels.py tests/test_capi.py -k "persistent_whole_k or tune" > "$OUT/gemm.out" 2>&1
rc=$?; echo "gemm rc=$rc"; tail -2 "$OUT/gemm.out"; [ $rc -le 1 ] || exit $rc
run eager_noprefix VGGT_ALIGN_GRAPH=0 VGGT_ALIGN_PREFIX=0 && run eager VGGT_ALIGN_GRAPH=0 && run graph VGGT_ALIGN_GRAPH=1
