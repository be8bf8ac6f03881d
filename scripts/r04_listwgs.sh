#!/bin/bash
# EXPERIMENT: list-role workgroups 128 (default) vs 256 / 512 (experiment build, same box)
set -o pipefail
mkdir -p gpurun_out
B="--steps 200 --warmup 30 --no-cpu-baseline"
for rep in 1 2; do
  for w in 128 256 512; do
    TT_EXPERIMENT_LIB=1 TT_LIST_WGS=$w timeout -k 10 240 python -u bench.py $B --ids zipf > gpurun_out/lw_z_${w}_$rep.log 2>&1 || exit 1
    echo "zipf wgs $w: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/lw_z_${w}_$rep.log)"
  done
  for w in 128 512; do
    TT_EXPERIMENT_LIB=1 TT_LIST_WGS=$w timeout -k 10 240 python -u bench.py $B > gpurun_out/lw_u_${w}_$rep.log 2>&1 || exit 1
    echo "uniform wgs $w: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/lw_u_${w}_$rep.log)"
  done
done
