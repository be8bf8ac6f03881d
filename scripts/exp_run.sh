set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline --ids zipf > gpurun_out/r02e_bench_zipf.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload config2 > gpurun_out/r02e_bench_config2.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --sharded > gpurun_out/r02e_bench_sharded_w1.log 2>&1 || exit $?
