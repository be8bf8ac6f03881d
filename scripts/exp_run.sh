set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ring.py tests/test_gpu_baseline_parity.py tests/test_gpu_step.py tests/test_gpu_dedup.py > gpurun_out/t_q.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_q.log 2>&1 || exit $?
TT_T1X=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_old.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/t1_stamps.py > gpurun_out/t1s.log 2>&1 || exit $?
