# Round-6 evidence, part A (each step time-limited, nothing more after a failure): the GPU suite as
# the driver runs it, smoke, the PMC passes (summary into profiles/ so the bench line carries its
# traffic), the default bench line (with the CPU leg) and the driver's short form.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r06x}
F=gpurun_out/$T
mkdir -p $F
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 170 --timeout-method thread > $F/gpu_tests.log 2>&1; rc=$?
echo "pytest exit=$rc" >> $F/gpu_tests.log; tail -3 $F/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || exit $?
tail -1 $F/smoke.log
OUT=gpurun_out/pmc_$T bash scripts/pmc_traffic.sh > $F/pmc.log 2>&1 || exit $?
cp gpurun_out/pmc_$T/summary.json profiles/${T}_pmc_traffic.json
cp gpurun_out/pmc_$T/summary.json $F/pmc_traffic.json
timeout -k 10 600 python bench.py > $F/bench.log 2>&1 || exit $?
tail -c 300 $F/bench.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $F/bench_driverlike.log 2>&1 || exit $?
echo "part A ok"
