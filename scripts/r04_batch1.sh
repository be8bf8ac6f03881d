# round 4: RMW / pooling probes, sharded KJT tests + bench, config-5 single-GPU kernel timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/profc5
timeout -k 10 120 ./scripts/micro_rmw.bin > gpurun_out/micro_rmw.log 2>&1 || exit $?
cat gpurun_out/micro_rmw.log
timeout -k 10 200 python scripts/pool_probe.py > gpurun_out/pool_probe.log 2>&1 || exit $?
cat gpurun_out/pool_probe.log | grep pooled
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded_kjt.py -x -q --timeout 240 --timeout-method thread > gpurun_out/skjt_tests.log 2>&1 || { tail -30 gpurun_out/skjt_tests.log; exit 1; }
tail -1 gpurun_out/skjt_tests.log
timeout -k 10 300 python bench.py --workload config5 --sharded --steps 30 --warmup 5 > gpurun_out/bench_c5_sharded_w1.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c5_sharded_w1.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profc5 -o c5 --output-format csv -- python3 bench.py --workload config5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/profc5.log 2>&1 || exit $?
python scripts/timeline.py gpurun_out/profc5/c5_kernel_trace.csv tower_l2_kernel 10 > gpurun_out/c5_timeline.txt 2>&1
head -20 gpurun_out/c5_timeline.txt
