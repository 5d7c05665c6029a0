# round 6, first lease: new tests (RCCL world-1 gather, close-then-reuse, 154x518 ATE/RPE), box baseline
# (headline bench), the alignment step's 6,608-row GEMMs vs hipBLASLt, align_chunk alone
set -u
O=gpurun_out/r11a; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_pipeline.py tests/test_gpu_fullsize.py::test_vkitti_sequence_ate_rpe_parity > $O/pytest.log 2>&1; rc=$?
echo pytest=$rc; grep -E "PASS|FAIL|ERROR|rel|ATE|hip" $O/pytest.log | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
tail -1 $O/bench.json | cut -c1-400
timeout -k 10 300 python -u scripts/gemmbench.py --tokens 6608 --shapes qkv,proj,fc1,fc2 --epis torch,plain,gelu --modes -1 > $O/gemm6608.txt 2>&1 || exit $?
grep -v '^{' $O/gemm6608.txt
timeout -k 10 300 python -u scripts/align_prof.py --reps 30 > $O/align.json 2>&1 || exit $?
tail -1 $O/align.json | cut -c1-600
