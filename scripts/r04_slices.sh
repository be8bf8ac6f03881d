#!/bin/bash
# EXPERIMENT: T2 slice depth (the slab rows T3 sums) 32 vs 16 vs 8 at the north star (experiment build)
set -o pipefail
mkdir -p gpurun_out
for p in 1 2 4 1 2 4; do
  TT_EXPERIMENT_LIB=1 TT_T2_SLICE_PASSES=$p timeout -k 10 240 python -u bench.py --steps 200 --warmup 30 > gpurun_out/slices_$p.log 2>&1 || exit 1
  echo "passes $p: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/slices_$p.log)"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for p in 1 2; do
rm -rf gpurun_out/slices_prof_$p
TT_EXPERIMENT_LIB=1 TT_T2_SLICE_PASSES=$p timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/slices_prof_$p -o run -- python3 bench.py --steps 100 --warmup 20 > gpurun_out/slices_prof_$p.log 2>&1 || exit 1
done
