# A/B on one box: the previous release library (lib_prev/, copied in before the call) against the
# tree's, interleaved 100-step bench runs; then targeted tests on the tree's library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["roofline"]["kernels"] if d.get("roofline") else {}
t = lambda n: k[n]["ms"] * 1e3 if n in k and k[n].get("ms") else float("nan")
print(f"{sys.argv[2]:>5} step {d['ms_per_step']*1e3:.2f} us  t1 {t('t1'):.2f}  tail {t('tail'):.2f}  t3 {t('t3'):.2f}", flush=True)
PY
}
# ORDER="new prev" runs the tree's library first in each pair; AA=1 runs lib_prev on both sides
# (an A/A: the noise floor and any bias of the run order)
for i in 1 2 3; do
  for v in ${ORDER:-prev new}; do
    if [ $v = prev ] || [ "${AA:-0}" = 1 ]; then L="TT_EXPERIMENT_LIB=$PWD/two_tower_recommender_model_amd/lib_prev/libtt_mi355x.so"; else L=""; fi
    env $L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 20 ${BENCH_ARGS:-} > $O/${v}_$i.log 2>&1 || exit $?
    summ $O/${v}_$i.log $v || exit $?
  done
done
