# Round 6: same-box A/B of a bench line between libraries (VARS: prev = lib_prev/, new = the tree's,
# exp = lib_exp/, other = lib_var/<name>/), R interleaved rounds; prints ms per step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06e}_ab
mkdir -p $O
P=$PWD/two_tower_recommender_model_amd
for i in $(seq 1 ${R:-3}); do
  for v in ${VARS:-prev new}; do
    case $v in
      prev) L="TT_EXPERIMENT_LIB=$P/lib_prev/libtt_mi355x.so" ;;
      new) L="" ;;
      exp) L="TT_EXPERIMENT_LIB=1" ;;
      *) L="TT_EXPERIMENT_LIB=$P/lib_var/$v/libtt_mi355x.so" ;;
    esac
    env $L timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-100} --warmup 20 ${BENCH_ARGS:---sharded} > $O/${v}_$i.log 2>&1 || exit $?
    python -c "
import json; d = json.loads([l for l in open('$O/${v}_$i.log') if l.startswith('{')][-1])
print('$v', round(d['ms_per_step'] * 1e3, 2), 'us', flush=True)" || exit $?
  done
done
