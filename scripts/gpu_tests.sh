set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest exit=$rc" >> gpurun_out/gpu_tests.log
tail -40 gpurun_out/gpu_tests.log
exit $rc
