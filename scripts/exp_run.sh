set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b_ns.log 2>&1 || exit $?
for v in 1 0 1 0; do
  TT_KJT_UPDATE_FIRST=$v timeout -k 10 300 python3 bench.py --workload config5 --steps 30 --warmup 5 --no-cpu-baseline >> gpurun_out/b_c5.log 2>&1 || exit $?
done
timeout -k 10 200 python3 scripts/t2_stamps.py > gpurun_out/t2_stamps.log 2>&1 || exit $?
