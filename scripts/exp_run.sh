set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/short_run_ramp.py > gpurun_out/ramp.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench_d1.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_d0.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench_d2.log 2>&1 || exit $?
