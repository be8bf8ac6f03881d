set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=two_tower_recommender_model_amd/lib/libtt_mi355x.so
for r in 1 2 3; do for v in 8 cs; do
cp gpu_ab_$v.so $L && timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_u_${v}_$r.log 2>&1 || exit $?
cp gpu_ab_$v.so $L && timeout -k 10 300 python -u bench.py --no-cpu-baseline --ids zipf > gpurun_out/bench_z_${v}_$r.log 2>&1 || exit $?
done; done
