set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2; do
TT_KJT_POOL_IN_T1=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload config5 > gpurun_out/bench_c5_off$i.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload config5 > gpurun_out/bench_c5_on$i.log 2>&1 || exit $?
done
mkdir -p gpurun_out/prof_c5off
TT_KJT_POOL_IN_T1=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5off -o c5 --output-format csv -- python3 bench.py --no-cpu-baseline --workload config5 --steps 30 > gpurun_out/prof_c5.log 2>&1 || exit $?
