# round 6: the asynchronous-ring attention (variant 10273): correctness first (bounded waits -- a lost
# signal gives wrong output, not a hang), then an interleaved in-model A/B against the new default
# (33 -> 2081 in the 8-wave form); then the whole GPU suite on the new default
set -u
O=gpurun_out/r11e; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "10273" > $O/pytest_10273.log 2>&1 || { tail -30 $O/pytest_10273.log; exit 1; }
tail -1 $O/pytest_10273.log
for r in 1 2; do
  for v in 33 10273; do
    VGGT_ATTN_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_v${v}_$r.json 2> $O/bench_v${v}_$r.err || exit $?
    python - $O/bench_v${v}_$r.json $v <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("variant", sys.argv[2], "ms/step", d["ms_per_step"], "attn frac", d["roofline"]["frac"], "attn us", round(1.9796e6/d["roofline"]["achieved"],1))
PY
  done
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; exit $rc
