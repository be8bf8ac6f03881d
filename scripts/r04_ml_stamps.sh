#!/bin/bash
# tail per-role timelines with the list role (experiment build) + kernel trace of the graph run
set -o pipefail
mkdir -p gpurun_out
TT_EXPERIMENT_LIB=1 TT_MULTI_LIST=1 K3_DD=192 timeout -k 10 180 python -u scripts/ring_stamps.py > gpurun_out/ml_stamps_on.log 2>&1 && \
GRAPH=1 TT_EXPERIMENT_LIB=1 TT_MULTI_LIST=1 K3_DD=192 timeout -k 10 180 python -u scripts/ring_stamps.py > gpurun_out/ml_stamps_on_g.log 2>&1 && \
GRAPH=1 TT_EXPERIMENT_LIB=1 TT_MULTI_LIST=0 timeout -k 10 180 python -u scripts/ring_stamps.py > gpurun_out/ml_stamps_off_g.log 2>&1 || exit 1
grep -hv amdgpu.ids gpurun_out/ml_stamps_on.log gpurun_out/ml_stamps_on_g.log gpurun_out/ml_stamps_off_g.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/mlp_on
TT_MULTI_LIST=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/mlp_on -o run -- python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/mlp_on.log 2>&1
