# A/B: T3 prefetch touching 1 or 2 segments per row (TLB + first lines) vs none (experiment library)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export TT_EXPERIMENT_LIB=1
for cfg in nopf seg1 seg2 nopf2; do
  case $cfg in
    nopf|nopf2) export TT_PREFETCH_NEXT=0; unset TT_PF_SEGS;;
    seg1) unset TT_PREFETCH_NEXT; export TT_PF_SEGS=1;;
    seg2) unset TT_PREFETCH_NEXT; export TT_PF_SEGS=2;;
  esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$cfg -o k --output-format csv -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab_prof_$cfg.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/ab_$cfg.log 2>&1 || exit $?
done
