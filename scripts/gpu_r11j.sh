# round 6: priority by the workgroup CU slot (HW_ID.TG_ID) for the 8-wave attention (variants 18465 / 34849)
set -u
O=gpurun_out/r11j; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "18465 or 34849" > $O/pytest_prio.log 2>&1 || { tail -30 $O/pytest_prio.log; exit 1; }
tail -1 $O/pytest_prio.log
for r in 1 2; do
  for v in 33 18465 34849; do
    VGGT_ATTN_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_v${v}_$r.json 2> $O/bench_v${v}_$r.err || exit $?
    python - $O/bench_v${v}_$r.json $v <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("variant", sys.argv[2], "ms/step", d["ms_per_step"], "attn frac", d["roofline"]["frac"], "attn us", round(1.9796e6/d["roofline"]["achieved"],1))
PY
  done
done
