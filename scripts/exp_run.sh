set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_round.sh || exit $?
OUT=gpurun_out/pmc_ns bash scripts/pmc_traffic.sh > gpurun_out/pmc_ns.log 2>&1 || exit $?
