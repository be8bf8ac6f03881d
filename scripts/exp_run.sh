set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || exit $?
for v in 0 1 0 1; do
  TT_EXPERIMENT_LIB=$v timeout -k 10 300 python3 bench.py --workload config5 --steps 32 --warmup 4 --no-cpu-baseline >> gpurun_out/ab_c5g.log 2>&1 || exit $?
done
for v in 0 1; do
  TT_EXPERIMENT_LIB=$v timeout -k 10 300 python3 bench.py --workload config5 --ids zipf --steps 32 --warmup 4 --no-cpu-baseline >> gpurun_out/ab_c5gz.log 2>&1 || exit $?
done
