#!/bin/bash
# EXPERIMENT (timing only): the Zipf tail's roles with the hot role / the slot role skipped
set -o pipefail
mkdir -p gpurun_out
for k in 0 1 2 3; do
GRAPH=1 IDS=zipf TT_EXP_SKIP=$k TT_EXPERIMENT_LIB=1 K3_DD=192 timeout -k 10 180 python -u scripts/ring_stamps.py > gpurun_out/zp_$k.log 2>&1 || exit 1
echo "== skip $k"; grep -v amdgpu.ids gpurun_out/zp_$k.log | grep "^tail" | head -2 | sed 's/slots\[385:513\] start [-0-9.]*\//slots start max /'
done
