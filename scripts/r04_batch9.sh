# config 5: two graph branches per step (one side stream) vs four — parity (bitwise tests) + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TT_KJT_BRANCHES=2 timeout -k 10 500 python -u -m pytest tests/test_gpu_multihot.py -x -q --timeout 250 --timeout-method thread > gpurun_out/mh2_tests.log 2>&1; tail -3 gpurun_out/mh2_tests.log | grep -E "passed|failed"
for i in 1 2; do
  TT_KJT_BRANCHES=2 timeout -k 10 300 python bench.py --workload config5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/c5_b2_$i.log 2>&1 || exit 1
  echo "2 branches $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5_b2_$i.log)"
  timeout -k 10 300 python bench.py --workload config5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/c5_b4_$i.log 2>&1 || exit 1
  echo "4 branches $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5_b4_$i.log)"
done
