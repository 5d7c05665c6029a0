# round 6, final: the RCCL self-P2P baton test alone (bounded), then the whole GPU suite, smoke, headline
set -u
O=gpurun_out/r11x; mkdir -p $O
timeout -k 10 150 python -u -m pytest -x -v -s --timeout 100 --timeout-method thread -m gpu \
  tests/test_gpu_pipeline.py::test_baton_p2p_batch_over_rccl_self > $O/pytest_p2p.log 2>&1; rc=$?
echo p2p=$rc; grep -E "PASSED|FAILED|Error|error" $O/pytest_p2p.log | head -5
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r11z.sh r11x tests,smoke,head
