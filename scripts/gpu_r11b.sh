# round 6: full-depth headline parity, ATE/RPE + frame_se3 bars at 1e-3, attention variant 545
# (3 K|V slots, DMA two tiles ahead) correctness, then an interleaved in-model A/B against variant 33
set -u
O=gpurun_out/r11b; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_fullsize.py \
  tests/test_gpu_model.py tests/test_gpu_ref_alignment.py > $O/pytest_parity.log 2>&1; rc=$?
echo parity=$rc; grep -E "PASSED|FAILED|full depth|hip vs|ATE|rmse|Error" $O/pytest_parity.log | cut -c1-300 | tail -60
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "545 or attention_eight_wave" > $O/pytest_attn.log 2>&1 || { tail -30 $O/pytest_attn.log; exit 1; }
tail -2 $O/pytest_attn.log
for r in 1 2; do
  for v in 33 545; do
    VGGT_ATTN_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_v${v}_$r.json 2> $O/bench_v${v}_$r.err || exit $?
    python - $O/bench_v${v}_$r.json $v <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("variant", sys.argv[2], "ms/step", d["ms_per_step"], "attn frac", d["roofline"]["frac"], "attn us", round(1.9796e6/d["roofline"]["achieved"],1))
PY
  done
done
