set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=two_tower_recommender_model_amd/lib/libtt_mi355x.so
for r in 1 2 3; do for v in base p1 p3; do
cp gpu_ab_$v.so $L && timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_u_${v}_$r.log 2>&1 || exit $?
done; done
for v in base p1 p3; do
cp gpu_ab_$v.so $L && timeout -k 10 300 python -u bench.py --no-cpu-baseline --ids zipf > gpurun_out/bench_z_${v}_1.log 2>&1 || exit $?
done
cp gpu_ab_p3.so $L && timeout -k 10 200 python -u scripts/ring_stamps.py > gpurun_out/rs_p3.log 2>&1 || exit $?
cp gpu_ab_base.so $L
