#!/bin/bash
# last check of the round's tree: the GPU suite + smoke, then the default bench line
set -o pipefail
sed -i 's/r04_gpu_suite_final3/r04_gpu_suite_final4/; s/r04_smoke3/r04_smoke4/' scripts/r04_suite.sh
bash scripts/r04_suite.sh || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r04d_bench.log 2>&1 || { tail -20 gpurun_out/r04d_bench.log; exit 1; }
tail -1 gpurun_out/r04d_bench.log | cut -c1-300
