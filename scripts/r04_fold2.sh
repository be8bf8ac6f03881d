#!/bin/bash
# T3 + T1 fold with the spread sense-reversal barrier: parity, then A/B bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ring.py tests/test_gpu_sharded.py -k "folded" > gpurun_out/fold2_test.log 2>&1 || { tail -40 gpurun_out/fold2_test.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/fold2_test.log | tail -6
timeout -k 10 240 python -u bench.py --steps 200 --warmup 30 > gpurun_out/fold2_off.log 2>&1 && \
TT_T1_FUSE=1 timeout -k 10 240 python -u bench.py --steps 200 --warmup 30 > gpurun_out/fold2_on.log 2>&1 && \
timeout -k 10 240 python -u bench.py --steps 200 --warmup 30 > gpurun_out/fold2_off2.log 2>&1 && \
TT_T1_FUSE=1 timeout -k 10 240 python -u bench.py --steps 200 --warmup 30 > gpurun_out/fold2_on2.log 2>&1 || exit 1
grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/fold2_off.log gpurun_out/fold2_on.log gpurun_out/fold2_off2.log gpurun_out/fold2_on2.log
