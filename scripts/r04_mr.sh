#!/bin/bash
# multi-lookup rows: 12 gradient rows in flight per half-wave (release) vs 4 (experiment build, -DDD_MR=4)
set -o pipefail
mkdir -p gpurun_out
true
true
B="--steps 200 --warmup 30 --no-cpu-baseline"
for rep in 1 2; do
  TT_EXPERIMENT_LIB=$PWD/two_tower_recommender_model_amd/lib_exp_a/libtt_mi355x.so timeout -k 10 240 python -u bench.py $B --ids zipf > gpurun_out/mr4_z_$rep.log 2>&1 && \
  TT_EXPERIMENT_LIB=1 timeout -k 10 240 python -u bench.py $B --ids zipf > gpurun_out/mr12_z_$rep.log 2>&1 && \
  TT_EXPERIMENT_LIB=$PWD/two_tower_recommender_model_amd/lib_exp_a/libtt_mi355x.so timeout -k 10 240 python -u bench.py $B > gpurun_out/mr4_u_$rep.log 2>&1 && \
  TT_EXPERIMENT_LIB=1 timeout -k 10 240 python -u bench.py $B > gpurun_out/mr12_u_$rep.log 2>&1 || exit 1
done
for f in mr4_z_1 mr12_z_1 mr4_z_2 mr12_z_2 mr4_u_1 mr12_u_1 mr4_u_2 mr12_u_2; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log)"; done
