#!/bin/bash
# tail per-role timelines (experiment build): list role on (default) / off, uniform / Zipf, the last
# tail of 8-step graph replays
set -o pipefail
mkdir -p gpurun_out
GRAPH=1 TT_EXPERIMENT_LIB=1 K3_DD=192 timeout -k 10 180 python -u scripts/ring_stamps.py > gpurun_out/ml_stamps_on_g.log 2>&1 && \
GRAPH=1 TT_EXPERIMENT_LIB=1 TT_MULTI_LIST=0 timeout -k 10 180 python -u scripts/ring_stamps.py > gpurun_out/ml_stamps_off_g.log 2>&1 && \
GRAPH=1 IDS=zipf TT_EXPERIMENT_LIB=1 K3_DD=192 timeout -k 10 180 python -u scripts/ring_stamps.py > gpurun_out/ml_stamps_zon_g.log 2>&1 || exit 1
grep -hv amdgpu.ids gpurun_out/ml_stamps_on_g.log gpurun_out/ml_stamps_off_g.log gpurun_out/ml_stamps_zon_g.log
