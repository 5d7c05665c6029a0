set -e
for L in old mi355x old mi355x; do
  echo $L; VGGT_MI355X_LIB=$PWD/large-scale-vit-slam_amd/lib/libvggt_$L.so timeout -k 10 200 python -u scripts/kbench.py --only gemm,norm --gemm-modes -1 --reps 30 > gpurun_out/ab_$L.log 2>&1
  tail -1 gpurun_out/ab_$L.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: v.get('us') for k, v in d.items() if 'qkv' in k or 'norm' in k or 'rope' in k})"
done
