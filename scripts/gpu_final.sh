# Round-end evidence: smoke, PMC passes (summary copied into profiles/ on the box so the bench line
# carries its traffic), the default bench line, the other workloads, a rocprofv3 kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
F=gpurun_out/final
mkdir -p $F
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || exit $?
OUT=gpurun_out/pmc bash scripts/pmc_traffic.sh > $F/pmc.log 2>&1 || exit $?
cp gpurun_out/pmc/summary.json profiles/${TAG:-r03u}_pmc_traffic.json
timeout -k 10 600 python bench.py > $F/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --ids zipf --no-cpu-baseline > $F/bench_zipf.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload config2 --no-cpu-baseline > $F/bench_config2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --sharded --no-cpu-baseline > $F/bench_sharded_w1.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --workload config5 --steps 30 --warmup 5 > $F/bench_config5.log 2>&1 || exit $?
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > $F/prof_bench.log 2>&1 || exit $?
