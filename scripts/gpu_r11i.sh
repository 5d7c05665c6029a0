# round 6: re-check after removing rejected attention variants -- attention tests, the counter passes on the
# final sources (fingerprint), the headline line
set -u
O=gpurun_out/r11i; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_aggregator.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash scripts/gpu_r11z.sh r11i pmc,head
