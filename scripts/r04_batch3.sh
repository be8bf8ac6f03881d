# round 4: T3 folded into T1 (ring + sharded), 64-wide row-owned T1 (config 2), hot-row teams by lookup share (Zipf) — parity, A/B bench, trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_t1f
timeout -k 10 500 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_dedup.py tests/test_gpu_sharded.py -x -v --timeout 200 --timeout-method thread -k "ring or dedup or folded or pipelined or w1_equals" > gpurun_out/t1f_tests.log 2>&1 || { tail -40 gpurun_out/t1f_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/t1f_tests.log | tail -3
timeout -k 10 300 python -u -m pytest tests/test_gpu_baseline_parity.py -x -v --timeout 250 --timeout-method thread -k "config2" > gpurun_out/c2_parity.log 2>&1 || { tail -40 gpurun_out/c2_parity.log; exit 1; }
grep -E "passed|failed" gpurun_out/c2_parity.log | tail -2
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_t1f.log 2>&1 || { tail -20 gpurun_out/bench_t1f.log; exit 1; }
tail -1 gpurun_out/bench_t1f.log | cut -c1-300
TT_T1_FUSE=0 timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_t1f_off.log 2>&1 || exit 1
tail -1 gpurun_out/bench_t1f_off.log | cut -c1-300
timeout -k 10 300 python bench.py --ids zipf --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_zipf.log 2>&1 || exit 1
tail -1 gpurun_out/bench_zipf.log | cut -c1-300
timeout -k 10 300 python bench.py --workload config2 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c2.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_t1f -o t1f --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof_t1f.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --sharded --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_sharded_w1.log 2>&1 || exit 1
tail -1 gpurun_out/bench_sharded_w1.log | cut -c1-300
