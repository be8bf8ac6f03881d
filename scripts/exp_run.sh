set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=two_tower_recommender_model_amd/lib/libtt_mi355x.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ring.py tests/test_gpu_baseline_parity.py > gpurun_out/t_tail.log 2>&1 || exit $?
IDS=zipf timeout -k 10 200 python -u scripts/ring_stamps.py > gpurun_out/rs_zipf.log 2>&1 || exit $?
for i in 1 2; do
for w in u z; do
A=""; [ $w = z ] && A="--ids zipf"
cp gpu_ab_old.so $L && timeout -k 10 300 python -u bench.py --no-cpu-baseline $A > gpurun_out/bench_${w}_old_$i.log 2>&1 || exit $?
cp gpu_ab_new.so $L && timeout -k 10 300 python -u bench.py --no-cpu-baseline $A > gpurun_out/bench_${w}_new_$i.log 2>&1 || exit $?
cp gpu_ab_new.so $L && TT_TAIL_HOT_WGS=64 timeout -k 10 300 python -u bench.py --no-cpu-baseline $A > gpurun_out/bench_${w}_n64_$i.log 2>&1 || exit $?
done
done
