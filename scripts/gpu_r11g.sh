# round 6: the alignment step's 6,608-row GEMM shapes -- every tile form of gemm_bf16
# against hipBLASLt (torch.matmul) on the same operands, plain / GELU / LayerScale-residual epilogues
set -u
O=gpurun_out/r11g; mkdir -p $O
timeout -k 10 600 python -u scripts/gemmbench.py --tokens 6608 --shapes qkv,proj,fc1,fc2 --epis torch,plain,gelu,resid \
  --modes=-1,0,1,2,3,4,5,6,7,8,9 --reps 50 > $O/gemm6608_modes.txt 2>&1 || { tail -20 $O/gemm6608_modes.txt; exit 1; }
grep -v '^{' $O/gemm6608_modes.txt | grep -v amdgpu.ids
