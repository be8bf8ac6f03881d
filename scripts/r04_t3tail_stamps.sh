#!/bin/bash
# per-role timelines of the tail launch with and without T3 inside it (experiment build)
set -o pipefail
mkdir -p gpurun_out
TT_EXPERIMENT_LIB=1 timeout -k 10 180 python -u scripts/ring_stamps.py > gpurun_out/t3tail_stamps_off.log 2>&1 && \
TT_EXPERIMENT_LIB=1 TT_T3_IN_TAIL=1 timeout -k 10 180 python -u scripts/ring_stamps.py > gpurun_out/t3tail_stamps_on.log 2>&1
rc=$?
cat gpurun_out/t3tail_stamps_off.log gpurun_out/t3tail_stamps_on.log | grep -v amdgpu.ids
exit $rc
