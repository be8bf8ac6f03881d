set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ns bash scripts/pmc_traffic.sh > gpurun_out/pmc_ns.log 2>&1 || exit $?
OUT=gpurun_out/pmc_c5 BENCH_ARGS="--workload config5" bash scripts/pmc_traffic.sh > gpurun_out/pmc_c5.log 2>&1 || exit $?
