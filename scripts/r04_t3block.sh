#!/bin/bash
# EXPERIMENT: T3 (tower_update_kernel) in 128-thread workgroups (388) vs 256 (194), experiment build
set -o pipefail
mkdir -p gpurun_out
B="--steps 200 --warmup 30 --no-cpu-baseline"
for rep in 1 2; do
  for bs in 256 128; do
    TT_EXPERIMENT_LIB=1 TT_T3_BLOCK=$bs timeout -k 10 240 python -u bench.py $B > gpurun_out/t3b_${bs}_$rep.log 2>&1 || exit 1
    echo "t3 block $bs: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/t3b_${bs}_$rep.log)"
  done
done
