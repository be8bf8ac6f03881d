# Round 6: the device-initiated exchange as the sharded default (self-test, direct stores by the
# producers, system-scope branch) — targeted GPU tests, then world-1 sharded bench lines A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r06a}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread ${TESTS:-tests/test_gpu_peer.py tests/test_gpu_sharded.py tests/test_gpu_multiproc_rehearsal.py tests/test_gpu_dropin_sharded.py} > gpurun_out/${T}_tests.log 2>&1; rc=$?
echo "pytest exit=$rc" >> gpurun_out/${T}_tests.log
tail -30 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for ex in ${EXCH:-auto rccl}; do
  timeout -k 10 240 python bench.py --sharded --exchange $ex --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/${T}_bench_sharded_$ex.log 2>&1 || exit $?
  tail -c 400 gpurun_out/${T}_bench_sharded_$ex.log; echo
done
TT_PEER_DIRECT=0 timeout -k 10 240 python bench.py --sharded --exchange peer --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/${T}_bench_sharded_peer_puts.log 2>&1 || exit $?
tail -c 400 gpurun_out/${T}_bench_sharded_peer_puts.log
