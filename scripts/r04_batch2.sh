# round 4: the ring with T3 folded into T1 — parity (ring tests), A/B bench, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_t1f
timeout -k 10 400 python -u -m pytest tests/test_gpu_ring.py -x -v --timeout 200 --timeout-method thread > gpurun_out/ring_tests.log 2>&1 || { tail -40 gpurun_out/ring_tests.log; exit 1; }
tail -3 gpurun_out/ring_tests.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_t1f.log 2>&1 || { tail -20 gpurun_out/bench_t1f.log; exit 1; }
tail -1 gpurun_out/bench_t1f.log | cut -c1-400
TT_T1_FUSE=0 timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_t1f_off.log 2>&1 || exit 1
tail -1 gpurun_out/bench_t1f_off.log | cut -c1-400
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_t1f_2.log 2>&1 || exit 1
tail -1 gpurun_out/bench_t1f_2.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_t1f -o t1f --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof_t1f.log 2>&1 || exit 1
ls gpurun_out/prof_t1f
