set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b_ns.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --sharded > gpurun_out/b_sh.log 2>&1 || exit $?
