set -u
O=gpurun_out/r1z; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_model.py > $O/pytest.log 2>&1; rc=$?; echo pytest=$rc; tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/sync_probe.py > $O/sync_probe.txt 2>&1 || exit $?; head -2 $O/sync_probe.txt | tail -1
timeout -k 10 400 python bench.py --workload chunk --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_chunk.json 2>&1 || exit $?; tail -1 $O/bench_chunk.json | cut -c1-200
timeout -k 10 400 python bench.py --workload train --steps 5 --warmup 2 > $O/bench_train.json 2>&1 || exit $?; tail -1 $O/bench_train.json | cut -c1-200
