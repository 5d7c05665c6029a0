set -u
O=gpurun_out/${1:-tr}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train.py > $O/pytest.log 2>&1; rc=$?; echo pytest=$rc; tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload train --steps 5 --warmup 2 > $O/bench_train.json 2>&1 || exit $?; tail -1 $O/bench_train.json | cut -c1-220
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/prof -o run -- python3 bench.py --workload train --steps 2 --warmup 1 > $O/prof.log 2>&1; echo prof=$?
