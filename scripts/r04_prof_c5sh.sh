set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/profc5sh
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profc5sh -o c5sh --output-format csv -- python3 bench.py --workload config5 --sharded --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/profc5sh.log 2>&1 || exit 1
tail -1 gpurun_out/profc5sh.log | cut -c1-120
python scripts/timeline.py gpurun_out/profc5sh/c5sh_kernel_trace.csv "kjt_route_count_kernel" 10 > gpurun_out/c5sh_timeline.txt 2>&1
head -30 gpurun_out/c5sh_timeline.txt
