# GPU suite, then (if green) the default bench line without the CPU leg; each step time-limited,
# nothing more after a failure. TAG names the logs: gpurun_out/$TAG_*.log
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-check}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 170 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${T}_tests.log 2>&1; rc=$?
echo "pytest exit=$rc" >> gpurun_out/${T}_tests.log
tail -15 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/${T}_bench.log 2>&1; rc=$?
echo "bench exit=$rc" >> gpurun_out/${T}_bench.log
tail -c 600 gpurun_out/${T}_bench.log
exit $rc
