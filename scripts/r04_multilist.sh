#!/bin/bash
# the tail's list role (TT_MULTI_LIST=1: T1 lists the multi-lookup rows and frees the single slots)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ring.py tests/test_gpu_baseline_parity.py tests/test_gpu_dedup.py > gpurun_out/ml_test0.log 2>&1 || { tail -40 gpurun_out/ml_test0.log; exit 1; }
TT_MULTI_LIST=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ring.py tests/test_gpu_baseline_parity.py > gpurun_out/ml_test.log 2>&1 || { tail -40 gpurun_out/ml_test.log; exit 1; }
grep -E "passed|failed" gpurun_out/ml_test0.log | tail -2
grep -E "passed|failed" gpurun_out/ml_test.log | tail -2
B="--steps 200 --warmup 30 --no-cpu-baseline"
for rep in 1 2; do
  timeout -k 10 240 python -u bench.py $B > gpurun_out/ml_off_$rep.log 2>&1 && \
  TT_MULTI_LIST=1 timeout -k 10 240 python -u bench.py $B > gpurun_out/ml_on_$rep.log 2>&1 && \
  timeout -k 10 240 python -u bench.py $B --ids zipf > gpurun_out/ml_zoff_$rep.log 2>&1 && \
  TT_MULTI_LIST=1 timeout -k 10 240 python -u bench.py $B --ids zipf > gpurun_out/ml_zon_$rep.log 2>&1 || exit 1
done
for f in ml_off_1 ml_on_1 ml_off_2 ml_on_2 ml_zoff_1 ml_zon_1 ml_zoff_2 ml_zon_2; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log)"; done
