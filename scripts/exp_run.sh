set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/s_bench.log 2>&1 || exit $?
TT_EXPERIMENT_LIB=1 timeout -k 10 300 python -u scripts/ring_stamps.py > gpurun_out/s_ring.log 2>&1 || exit $?
tail -2 gpurun_out/s_ring.log
timeout -k 10 300 python -u scripts/rows_stamps.py > gpurun_out/s_rows_stamps.log 2>&1 || exit $?
cat gpurun_out/s_rows_stamps.log
