#!/bin/bash
# the GPU suite as the driver runs it, then smoke()
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04_gpu_suite_final3.log 2>&1
rc=$?
tail -5 gpurun_out/r04_gpu_suite_final3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke3.log 2>&1; rc=$?
tail -2 gpurun_out/r04_smoke3.log
exit $rc
