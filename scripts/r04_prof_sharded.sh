set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/profsh
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profsh -o sh --output-format csv -- python3 bench.py --sharded --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/profsh.log 2>&1 || exit 1
python scripts/timeline.py gpurun_out/profsh/sh_kernel_trace.csv "tower_rows_kernel<false, true" 20 > gpurun_out/sh_timeline.txt 2>&1
head -20 gpurun_out/sh_timeline.txt
