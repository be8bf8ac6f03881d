# Round-6 evidence, part B: the other workload lines, the sharded and drop-in lines, a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r06x}
F=gpurun_out/$T
mkdir -p $F
timeout -k 10 300 python bench.py --ids zipf --no-cpu-baseline > $F/bench_idszipf.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload config2 --no-cpu-baseline > $F/bench_workloadconfig2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --sharded --no-cpu-baseline --steps 100 > $F/bench_sharded.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --sharded --exchange rccl --no-cpu-baseline --steps 100 > $F/bench_sharded_rccl.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --path dropin --no-cpu-baseline > $F/bench_pathdropin.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --workload config5 --steps 30 --warmup 5 --no-cpu-baseline > $F/bench_workloadconfig5.log 2>&1 || exit $?
mkdir -p gpurun_out/prof_$T
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o bench --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > $F/prof_bench.log 2>&1 || exit $?
find gpurun_out/prof_$T -name "*kernel_stats.csv" -exec cp {} $F/bench_kernel_stats.csv \;
echo "part B ok"
