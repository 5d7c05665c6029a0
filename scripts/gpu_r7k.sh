#!/bin/bash
# qkv-shaped GEMMs (N 3072: 1,032 tiles = 4 rounds + 8 at 256 rows) on 192-row tiles (6 rounds of 192): library
# built with -DVGGT_BM_RULE_LE against the default; GEMM tests on it first.  usage: TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
L=$PWD/large-scale-vit-slam_amd/lib
VGGT_MI355X_LIB=$L/libvggt_bmle.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "gemm" > "$OUT/pytest_bmle.log" 2>&1 || { tail -20 "$OUT/pytest_bmle.log"; exit 1; }
tail -1 "$OUT/pytest_bmle.log"
for b in 256 192; do
  VGGT_GEMM_BM=$b timeout -k 10 200 python3 -u scripts/pipebench.py --pipes 5 --rounds 2 > "$OUT/pb_bm$b.txt" 2>&1 || exit 1
  grep -E "^qkv" "$OUT/pb_bm$b.txt" | sed "s/^/bm$b /"
done
run() {  # name, bench args (quoted), env...
  local n=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py $args --no-cpu-baseline > "$OUT/$n.tmp" 2>> "$OUT/err.log" || exit $?
  cat "$OUT/$n.tmp" >> "$OUT/$n.json"
  echo "$n: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['value'])" "$OUT/$n.tmp")"
}
for r in 1 2; do
  run agg_def ""
  run agg_bmle "" VGGT_MI355X_LIB=$L/libvggt_bmle.so
done
run c3_def "--config 3 --steps 2 --warmup 1"
run c3_bmle "--config 3 --steps 2 --warmup 1" VGGT_MI355X_LIB=$L/libvggt_bmle.so
# the fused qkv GEMM on the whole-K-tile loop (VGGT_GEMM_FULLK=7)
VGGT_GEMM_FULLK=7 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "qkv" > "$OUT/pytest_fk7.log" 2>&1 || { tail -20 "$OUT/pytest_fk7.log"; exit 1; }
tail -1 "$OUT/pytest_fk7.log"
for r in 1 2; do
  for f in 5 7; do
    VGGT_GEMM_FULLK=$f timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$OUT/fk$f.tmp" 2>> "$OUT/bench_err.log" || exit $?
    cat "$OUT/fk$f.tmp" >> "$OUT/fk$f.json"
    echo "fullk $f: $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" "$OUT/fk$f.tmp")"
  done
done
# configs[3] kernel table with the current defaults
P=/tmp/prof_$1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $P/c3 -o run -- python3 bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_c3.log" 2>&1 || exit $?
python3 scripts/prof_summary.py $(find $P/c3 -name "*results.db" | head -1) > "$OUT/c3_kernels.md" || exit $?
head -30 "$OUT/c3_kernels.md"
