set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest exit=$rc" >> gpurun_out/gpu_tests.log
tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke exit=$?" >> gpurun_out/smoke.log
tail -5 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1; echo "bench exit=$?" >> gpurun_out/bench.log
tail -5 gpurun_out/bench.log
