#!/bin/bash
# New defaults (GEMM pipe 5 incl. the half-K loop, frame-only 16x16 attention): full GPU suite, GEMM timings,
# aggregator A/B against the r7b library.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
bash scripts/gpu_tests.sh "$1" || exit $?
timeout -k 10 240 python3 -u scripts/pipebench.py --pipes 0,5,13 > "$OUT/pipebench.txt" 2>&1 || { tail -5 "$OUT/pipebench.txt"; exit 1; }
grep -v bitwise "$OUT/pipebench.txt"
OLD=$PWD/large-scale-vit-slam_amd/lib/libvggt_r7b.so
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu-baseline > "$OUT/$n.tmp" 2>> "$OUT/err.log" || exit $?
  cat "$OUT/$n.tmp" >> "$OUT/$n.json"
  echo "$n: $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" "$OUT/$n.tmp")"
}
for r in 1 2; do
  run old VGGT_MI355X_LIB=$OLD VGGT_GEMM_PIPE=0 VGGT_ATTN16=0
  run new VGGT_GEMM_PIPE=5
  run new_p13 VGGT_GEMM_PIPE=13
done
