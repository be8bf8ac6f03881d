set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=two_tower_recommender_model_amd/lib/libtt_mi355x.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sharded.py tests/test_gpu_dmp.py tests/test_gpu_multiproc_rehearsal.py > gpurun_out/t_sg.log 2>&1 || exit $?
for i in 1 2 3; do
for v in old new; do
cp gpu_ab_$v.so $L && timeout -k 10 300 python -u bench.py --no-cpu-baseline --sharded --steps 50 > gpurun_out/bench_sh_${v}_$i.log 2>&1 || exit $?
done
done
cp gpu_ab_new.so $L
