#!/bin/bash
# kernel durations with and without the tail's list role
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/mlp_off gpurun_out/mlp_on
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/mlp_off -o run -- python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/mlp_off.log 2>&1 && \
TT_MULTI_LIST=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/mlp_on -o run -- python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/mlp_on.log 2>&1
