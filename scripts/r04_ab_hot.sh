# A/B on one box: ring with the hot rows in the T3 launch (default) vs in the tail (TT_HOT_IN_T3=0),
# Zipf and uniform ids; then the ring / dedup parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_dedup.py -x -q --timeout 200 --timeout-method thread > gpurun_out/hot_tests.log 2>&1 || { tail -40 gpurun_out/hot_tests.log; exit 1; }
tail -1 gpurun_out/hot_tests.log
for i in 1 2; do
  for ids in zipf uniform; do
    timeout -k 10 300 python bench.py --ids $ids --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/ab_t3_${ids}_$i.log 2>&1 || exit 1
    echo "hotT3 $ids $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_t3_${ids}_$i.log) $(grep -o '"event_span_ms": {[^}]*}' gpurun_out/ab_t3_${ids}_$i.log)"
    TT_HOT_IN_T3=0 timeout -k 10 300 python bench.py --ids $ids --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/ab_tail_${ids}_$i.log 2>&1 || exit 1
    echo "hotTail $ids $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_tail_${ids}_$i.log) $(grep -o '"event_span_ms": {[^}]*}' gpurun_out/ab_tail_${ids}_$i.log)"
  done
done
