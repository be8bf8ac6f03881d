#!/bin/bash
# EXPERIMENT: the ring tail's insert role at 1 lookup per thread (64 workgroups) vs 2 (32), experiment builds
set -o pipefail
mkdir -p gpurun_out
B="--steps 200 --warmup 30 --no-cpu-baseline"
A=$PWD/two_tower_recommender_model_amd/lib_exp_a/libtt_mi355x.so
timeout -k 10 300 env TT_EXPERIMENT_LIB=$A python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ring.py > gpurun_out/inspt_test.log 2>&1 || { tail -20 gpurun_out/inspt_test.log; exit 1; }
tail -1 gpurun_out/inspt_test.log
for rep in 1 2; do
  TT_EXPERIMENT_LIB=1 timeout -k 10 240 python -u bench.py $B > gpurun_out/ip2_u_$rep.log 2>&1 && \
  TT_EXPERIMENT_LIB=$A timeout -k 10 240 python -u bench.py $B > gpurun_out/ip1_u_$rep.log 2>&1 && \
  TT_EXPERIMENT_LIB=1 timeout -k 10 240 python -u bench.py $B --ids zipf > gpurun_out/ip2_z_$rep.log 2>&1 && \
  TT_EXPERIMENT_LIB=$A timeout -k 10 240 python -u bench.py $B --ids zipf > gpurun_out/ip1_z_$rep.log 2>&1 || exit 1
done
for f in ip2_u_1 ip1_u_1 ip2_u_2 ip1_u_2 ip2_z_1 ip1_z_1 ip2_z_2 ip1_z_2; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log)"; done
