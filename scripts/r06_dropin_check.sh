# Round 6: the N > 1 drop-in (agreed admission, KJT mode) as processes sharing the GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r06b}
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_dropin_sharded.py tests/test_gpu_multiproc_rehearsal.py::test_bench_dropin_config5_n2_dispatches_kjt_step tests/test_gpu_multiproc_rehearsal.py::test_bench_dropin_n2_rehearsal} > gpurun_out/${T}_tests.log 2>&1; rc=$?
echo "pytest exit=$rc" >> gpurun_out/${T}_tests.log
tail -40 gpurun_out/${T}_tests.log
exit $rc
