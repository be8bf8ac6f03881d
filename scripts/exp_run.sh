set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/t1_wave_stamps.py > gpurun_out/t1w.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_q.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/t_q.log 2>&1 || exit $?
