set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ring.py > gpurun_out/t_ring.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench_d1.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_d0.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench_d2.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 16 --warmup 8 > gpurun_out/bench_d3.log 2>&1 || exit $?
