# round 4: config 5 grouping joined by the next step's update (cross-step) — parity + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/profc5d
timeout -k 10 500 python -u -m pytest tests/test_gpu_multihot.py tests/test_gpu_baseline_parity.py -x -q --timeout 250 --timeout-method thread -k "multihot or config5" > gpurun_out/mh_tests.log 2>&1; tail -30 gpurun_out/mh_tests.log | grep -E "passed|failed|Error|assert" | tail -8
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload config5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/c5_x_$i.log 2>&1 || exit 1
  echo "crossstep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5_x_$i.log)"
  TT_KJT_CROSS_STEP=0 timeout -k 10 300 python bench.py --workload config5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/c5_nx_$i.log 2>&1 || exit 1
  echo "endjoin $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5_nx_$i.log)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profc5d -o c5x --output-format csv -- python3 bench.py --workload config5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/profc5d.log 2>&1 || exit 1
python scripts/timeline.py gpurun_out/profc5d/c5x_kernel_trace.csv tower_l2_kernel 10 > gpurun_out/c5x_timeline.txt 2>&1
head -16 gpurun_out/c5x_timeline.txt
