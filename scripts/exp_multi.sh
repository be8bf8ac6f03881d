# EXPERIMENT: several libraries round-robin on one box (interleaved 100-step bench runs, R rounds):
# VARS names libraries — "prev" (lib_prev/), "new" (the tree's lib/), "exp" (lib_exp/), anything else
# lib_var/<name>/; "<lib>+VAR=value" adds an environment setting to that run (e.g. exp+TT_DD_HOT_WGS=128)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/multi
mkdir -p $O
P=$PWD/two_tower_recommender_model_amd
for i in $(seq 1 ${R:-3}); do
  for v in ${VARS:-prev new}; do
    lib=${v%%+*}
    extra=""
    [ "$lib" != "$v" ] && extra=${v#*+}
    case $lib in
      prev) L="TT_EXPERIMENT_LIB=$P/lib_prev/libtt_mi355x.so" ;;
      new) L="" ;;
      exp) L="TT_EXPERIMENT_LIB=1" ;;
      *) L="TT_EXPERIMENT_LIB=$P/lib_var/$lib/libtt_mi355x.so" ;;
    esac
    L="$L $extra"
    env $L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 20 ${BENCH_ARGS:-} > "$O/${v//[+=]/_}_$i.log" 2>&1 || exit $?
    python - "$O/${v//[+=]/_}_$i.log" $v <<'PY' || exit $?
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["roofline"]["kernels"] if d.get("roofline") else {}
t = lambda n: k[n]["ms"] * 1e3 if n in k and k[n].get("ms") else float("nan")
print(f"{sys.argv[2]:>5} step {d['ms_per_step']*1e3:.2f} us  t1 {t('t1'):.2f}  tail {t('tail'):.2f}  t3 {t('t3'):.2f}", flush=True)
PY
  done
done
