set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=two_tower_recommender_model_amd/lib/libtt_mi355x.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ring.py tests/test_gpu_step.py tests/test_gpu_sharded.py tests/test_gpu_multihot.py tests/test_gpu_baseline_parity.py > gpurun_out/t_t3.log 2>&1 || exit $?
for i in 1 2 3; do
cp gpu_ab_old.so $L && timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_old_$i.log 2>&1 || exit $?
cp gpu_ab_new.so $L && timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_new_$i.log 2>&1 || exit $?
done
