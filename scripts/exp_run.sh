set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/profsh
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profsh -o sh --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --sharded > gpurun_out/p_prof_sh.log 2>&1 || exit $?
