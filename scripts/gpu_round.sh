# tests -> smoke -> bench -> rocprofv3 kernel stats (each step time-limited; stop at first hard failure)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest exit=$rc" >> gpurun_out/gpu_tests.log
tail -25 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi  # a failing test may be a GPU fault: run nothing more
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke exit=$rc" >> gpurun_out/smoke.log; tail -2 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?
echo "bench exit=$rc" >> gpurun_out/bench.log; tail -3 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof_bench.log 2>&1
echo "prof exit=$?" >> gpurun_out/prof_bench.log; tail -1 gpurun_out/prof_bench.log
