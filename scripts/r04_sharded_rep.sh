# the sharded world-1 bench three times (graph capture with RCCL inside): does the capture fail?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --sharded --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/sh_$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc $(grep -c 'capture with collectives refused' gpurun_out/sh_$i.log) refusals $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sh_$i.log) $(grep -o '"mode": "[a-z]*"' gpurun_out/sh_$i.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
