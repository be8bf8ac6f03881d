set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/ab_k2.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps-per-graph 8 >> gpurun_out/ab_k2.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --warmup 10 >> gpurun_out/ab_k2.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --warmup 10 --steps-per-graph 8 >> gpurun_out/ab_k2.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 >> gpurun_out/ab_k2.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 --steps-per-graph 8 >> gpurun_out/ab_k2.log 2>&1 || exit $?
