set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sharded.py > gpurun_out/t_q.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --sharded --steps 30 > gpurun_out/bench_sh1.log 2>&1 || exit $?
TT_U_DD_FIRST=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --sharded --steps 30 > gpurun_out/bench_sh0.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --sharded --steps 30 > gpurun_out/bench_sh1b.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/owner_update_stamps.py > gpurun_out/own.log 2>&1 || exit $?
