set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multihot.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || exit $?
for k in 8 1 8 1; do
  timeout -k 10 300 python3 bench.py --workload config5 --steps 32 --warmup 4 --no-cpu-baseline --steps-per-graph $k >> gpurun_out/ab_c5k.log 2>&1 || exit $?
done
