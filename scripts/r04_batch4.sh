# round 4: fold opt-in (off by default) — benches with the default ring: north star, Zipf (hot-row
# teams by lookup share), config 2 (64-wide row-owned T1), sharded world 1; fold tests (opt-in)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r04b
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_ns.log 2>&1 || { tail -20 gpurun_out/bench_ns.log; exit 1; }
tail -1 gpurun_out/bench_ns.log | cut -c1-200
timeout -k 10 300 python bench.py --ids zipf --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_zipf.log 2>&1 || exit 1
tail -1 gpurun_out/bench_zipf.log | cut -c1-200
timeout -k 10 300 python bench.py --workload config2 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c2.log | cut -c1-200
timeout -k 10 400 python bench.py --sharded --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_sharded_w1.log 2>&1 || exit 1
tail -1 gpurun_out/bench_sharded_w1.log | cut -c1-200
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread -k "folded" > gpurun_out/fold_tests.log 2>&1 || { tail -30 gpurun_out/fold_tests.log; exit 1; }
tail -1 gpurun_out/fold_tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04b -o c2 --output-format csv -- python3 bench.py --workload config2 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04b -o zipf --output-format csv -- python3 bench.py --ids zipf --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof_zipf.log 2>&1 || exit 1
ls gpurun_out/prof_r04b
