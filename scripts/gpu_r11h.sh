# round 6: the alignment step's fused GEMMs vs hipBLASLt + torch epilogues at 6,608 rows; the four-rank ring
# with the planner's own offload placement
set -u
O=gpurun_out/r11h; mkdir -p $O
timeout -k 10 300 python -u scripts/align_gemm_vs_hipblaslt.py > $O/align_gemm.txt 2>&1 || { tail -20 $O/align_gemm.txt; exit 1; }
grep -v '^{' $O/align_gemm.txt | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_ring.py > $O/pytest_ring.log 2>&1; rc=$?
grep -E "PASSED|FAILED|moved|rel-L2 vs the single-process loop [0-9.e-]+$" $O/pytest_ring.log | grep -E "PASSED|FAILED|moved|rank 0 pose" | head -20
exit $rc
