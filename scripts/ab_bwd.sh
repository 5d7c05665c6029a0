set -e
for L in old mi355x old mi355x; do
  echo $L; VGGT_MI355X_LIB=$PWD/large-scale-vit-slam_amd/lib/libvggt_$L.so timeout -k 10 120 python -u scripts/bwdbench.py | tail -1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train.py > gpurun_out/pt_train.log 2>&1; echo pytest=$?; tail -2 gpurun_out/pt_train.log
