# round 4: hot-row teams filed at insert time (one member per 96 lookups past 30) — parity + Zipf bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_dedup.py -x -q --timeout 200 --timeout-method thread > gpurun_out/hot_tests.log 2>&1 || { tail -40 gpurun_out/hot_tests.log; exit 1; }
tail -1 gpurun_out/hot_tests.log
timeout -k 10 300 python bench.py --ids zipf --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_zipf.log 2>&1 || exit 1
tail -1 gpurun_out/bench_zipf.log | cut -c1-200
grep -o '"event_span_ms": {[^}]*}' gpurun_out/bench_zipf.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_ns.log 2>&1 || exit 1
tail -1 gpurun_out/bench_ns.log | cut -c1-200
grep -o '"event_span_ms": {[^}]*}' gpurun_out/bench_ns.log
