# round 6: DPT pre-split convolution with a three-stage LDS ring (VGGT_CONV_STAGES=3) -- correctness under the
# knob, then isolated (convbench_pre) and in-model (full chunk, configs[3]) A/B against the double buffer
set -u
O=gpurun_out/r11k; mkdir -p $O
VGGT_CONV_STAGES=3 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_model.py -k "conv or dpt" > $O/pytest_conv3.log 2>&1 || { tail -30 $O/pytest_conv3.log; exit 1; }
tail -1 $O/pytest_conv3.log
for r in 1 2; do
  for st in 2 3; do
    VGGT_CONV_STAGES=$st timeout -k 10 300 python -u scripts/convbench_pre.py --reps 20 > $O/convbench_s${st}_$r.txt 2>&1 || exit $?
    echo "stages=$st"; grep -v amdgpu.ids $O/convbench_s${st}_$r.txt | tail -6
  done
done
for r in 1 2; do
  for st in 2 3; do
    VGGT_CONV_STAGES=$st timeout -k 10 300 python bench.py --workload chunk --steps 10 --warmup 3 --no-cpu-baseline > $O/chunk_s${st}_$r.json 2> $O/chunk_s${st}_$r.err || exit $?
    echo "stages=$st chunk ms/step $(python -c "import json,sys; print(json.loads(open('$O/chunk_s${st}_$r.json').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
