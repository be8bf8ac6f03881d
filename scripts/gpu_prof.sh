set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
echo "exit=$?" >> gpurun_out/prof_bench.log
tail -3 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*stats*" | head
