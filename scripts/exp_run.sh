set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_cols.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_cols.log 2>&1 || exit $?
for r in 1 2 3; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_u_s_$r.log 2>&1 || exit $?
TT_T3_VEC4=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_u_v_$r.log 2>&1 || exit $?
done
TT_T3_VEC4=1 timeout -k 10 200 python -u scripts/ring_stamps.py > gpurun_out/rs_v.log 2>&1 || exit $?
