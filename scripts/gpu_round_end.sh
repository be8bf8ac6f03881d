# Round-end evidence in one call, each step time-limited, nothing more after a failure: the GPU
# suite, smoke, PMC passes (summary into profiles/ on the box so the bench line carries its
# traffic), the default bench line (with the CPU leg), the other workloads, a rocprofv3 kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r05x}
F=gpurun_out/$T
mkdir -p $F
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 170 --timeout-method thread > $F/gpu_tests.log 2>&1; rc=$?
echo "pytest exit=$rc" >> $F/gpu_tests.log; tail -3 $F/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || exit $?
tail -1 $F/smoke.log
OUT=gpurun_out/pmc bash scripts/pmc_traffic.sh > $F/pmc.log 2>&1 || exit $?
cp gpurun_out/pmc/summary.json profiles/${T}_pmc_traffic.json
timeout -k 10 600 python bench.py > $F/bench.log 2>&1 || exit $?
tail -c 300 $F/bench.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $F/bench_driverlike.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --ids zipf --no-cpu-baseline > $F/bench_idszipf.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload config2 --no-cpu-baseline > $F/bench_workloadconfig2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --sharded --no-cpu-baseline > $F/bench_sharded.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --sharded --exchange peer --no-cpu-baseline > $F/bench_sharded_peer.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --path dropin --no-cpu-baseline > $F/bench_pathdropin.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --workload config5 --steps 30 --warmup 5 --no-cpu-baseline > $F/bench_workloadconfig5.log 2>&1 || exit $?
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > $F/prof_bench.log 2>&1 || exit $?
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} $F/bench_kernel_stats.csv \;
echo "round-end ok"
