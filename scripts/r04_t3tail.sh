#!/bin/bash
# T3 inside the tail launch: bitwise parity vs the three-launch ring, A/B bench, kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ring.py -k "t3_in_tail" > gpurun_out/t3tail_test.log 2>&1 || { tail -40 gpurun_out/t3tail_test.log; exit 1; }
tail -3 gpurun_out/t3tail_test.log
timeout -k 10 240 python -u bench.py --steps 200 --warmup 30 > gpurun_out/t3tail_off.log 2>&1 && \
TT_T3_IN_TAIL=1 timeout -k 10 240 python -u bench.py --steps 200 --warmup 30 > gpurun_out/t3tail_on.log 2>&1 && \
timeout -k 10 240 python -u bench.py --steps 200 --warmup 30 > gpurun_out/t3tail_off2.log 2>&1 && \
TT_T3_IN_TAIL=1 timeout -k 10 240 python -u bench.py --steps 200 --warmup 30 > gpurun_out/t3tail_on2.log 2>&1 || exit 1
grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/t3tail_off.log gpurun_out/t3tail_on.log gpurun_out/t3tail_off2.log gpurun_out/t3tail_on2.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/t3t_on
TT_T3_IN_TAIL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/t3t_on -o run -- python3 bench.py --steps 100 --warmup 20 > gpurun_out/t3t_prof_on.log 2>&1
