set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --sharded --steps 20 --warmup 5 > gpurun_out/bench_sh.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload config5 --steps 20 --warmup 5 > gpurun_out/bench_c5.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
