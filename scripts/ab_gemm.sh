set -e
mkdir -p gpurun_out/ab
for r in 1 2; do
for L in old mi355x; do
  VGGT_MI355X_LIB=$PWD/large-scale-vit-slam_amd/lib/libvggt_$L.so timeout -k 10 200 python -u scripts/kbench.py --only gemm --gemm-modes 0 --reps 30 > gpurun_out/ab/gemm_${L}_$r.log 2>&1
  echo "$L $r"; grep -E "^(proj|fc2)" gpurun_out/ab/gemm_${L}_$r.log
done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k gemm > gpurun_out/ab/pytest_gemm.log 2>&1; echo pytest=$?; tail -2 gpurun_out/ab/pytest_gemm.log
