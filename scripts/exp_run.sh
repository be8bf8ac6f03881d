set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=two_tower_recommender_model_amd/lib/libtt_mi355x.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ring.py tests/test_gpu_step.py tests/test_gpu_baseline_parity.py > gpurun_out/t_pf.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/ring_stamps.py > gpurun_out/rs_uniform.log 2>&1 || exit $?
for i in 1 2 3; do
for v in old new; do
cp gpu_ab_$v.so $L && timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 100 > gpurun_out/bench_u_${v}_$i.log 2>&1 || exit $?
done
done
cp gpu_ab_new.so $L
