# round 6: attention segment stamps, attention tests on the rebuilt library,
# the CPU baseline's thread-scaling curve (BASELINE.md §3 row C2, 4 / 8 / 16 threads)
set -u
O=gpurun_out/r11c; mkdir -p $O profiles/r11
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "attention" > $O/pytest_attn.log 2>&1 || { tail -30 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
timeout -k 10 300 python -u scripts/attn_stamps.py --out $O/attn_stamps_global.json > $O/attn_stamps_global.txt 2>&1 || { tail -20 $O/attn_stamps_global.txt; exit 1; }
cat $O/attn_stamps_global.json
timeout -k 10 300 python -u scripts/attn_stamps.py --tokens 1374 --batch 16 --out $O/attn_stamps_frame.json > $O/attn_stamps_frame.txt 2>&1 || { tail -20 $O/attn_stamps_frame.txt; exit 1; }
grep -A5 cycles_per_tile $O/attn_stamps_frame.json
timeout -k 10 600 python -u scripts/cpu_thread_scaling.py --out $O/cpu_thread_scaling.json > $O/cpu_thread_scaling.txt 2>&1 || { tail -20 $O/cpu_thread_scaling.txt; exit 1; }
grep threads= $O/cpu_thread_scaling.txt
