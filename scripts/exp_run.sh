set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread >> gpurun_out/gpu_suite.log 2>&1 || exit $?
for v in 0 1 0 1 0 1; do
  TT_EXPERIMENT_LIB=$v timeout -k 10 200 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline >> gpurun_out/ab_list.log 2>&1 || exit $?
done
for v in 0 1; do
  TT_EXPERIMENT_LIB=$v timeout -k 10 200 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --ids zipf >> gpurun_out/ab_list_z.log 2>&1 || exit $?
done
