# A/B on one box: Zipf ring step, hot-row teams filed at insert (lib) vs round-3 teams (lib_exp)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python bench.py --ids zipf --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/ab_new_$i.log 2>&1 || exit 1
  echo "new $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_new_$i.log) $(grep -o '"event_span_ms": {[^}]*}' gpurun_out/ab_new_$i.log)"
  TT_EXPERIMENT_LIB=1 timeout -k 10 300 python bench.py --ids zipf --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/ab_old_$i.log 2>&1 || exit 1
  echo "old $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_old_$i.log) $(grep -o '"event_span_ms": {[^}]*}' gpurun_out/ab_old_$i.log)"
done
