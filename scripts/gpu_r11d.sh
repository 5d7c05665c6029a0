# round 6: attention variants from the segment stamps -- 2081 (LDS-DMA issued by the priority half),
# 4129 (no priority raise): correctness, stamps, interleaved in-model A/B against 33
set -u
O=gpurun_out/r11d; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "attention" > $O/pytest_attn.log 2>&1 || { tail -30 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
for v in 33 2081 4129; do
  timeout -k 10 300 python -u scripts/attn_stamps.py --variant $v --out $O/attn_stamps_v$v.json > $O/attn_stamps_v$v.txt 2>&1 || { tail -20 $O/attn_stamps_v$v.txt; exit 1; }
  python - $O/attn_stamps_v$v.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print(d["variant"], "plain us", d["us_plain"], "stamped", d["us_stamped"], "per tile", d["cycles_per_tile"], "bar by slot", d["barrier_by_wave_slot"][0], d["barrier_by_wave_slot"][4], "work", d["work_by_wave_slot"][0], d["work_by_wave_slot"][4])
PY
done
for r in 1 2; do
  for v in 33 2081 4129; do
    VGGT_ATTN_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_v${v}_$r.json 2> $O/bench_v${v}_$r.err || exit $?
    python - $O/bench_v${v}_$r.json $v <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("variant", sys.argv[2], "ms/step", d["ms_per_step"], "attn frac", d["roofline"]["frac"], "attn us", round(1.9796e6/d["roofline"]["achieved"],1))
PY
  done
done
