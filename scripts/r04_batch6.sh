# round 4: pooled-input row-owned T1 (multi-hot path after tt_pooled_fwd) — parity + config 5 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/profc5b
timeout -k 10 500 python -u -m pytest tests/test_gpu_multihot.py tests/test_gpu_sharded_kjt.py -x -q --timeout 200 --timeout-method thread > gpurun_out/mh_tests.log 2>&1; tail -30 gpurun_out/mh_tests.log | grep -E "passed|failed|Error|assert" | tail -8
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload config5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/c5_fused_$i.log 2>&1 || exit 1
  echo "fusedpool $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5_fused_$i.log)"
  TT_KJT_POOL_IN_T1=0 timeout -k 10 300 python bench.py --workload config5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/c5_unfused_$i.log 2>&1 || exit 1
  echo "pooled+rowsT1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5_unfused_$i.log)"
done
TT_KJT_POOL_IN_T1=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profc5b -o c5u --output-format csv -- python3 bench.py --workload config5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/profc5b.log 2>&1 || exit 1
python scripts/timeline.py gpurun_out/profc5b/c5u_kernel_trace.csv pooled_fwd_kernel 10 > gpurun_out/c5u_timeline.txt 2>&1
head -16 gpurun_out/c5u_timeline.txt
