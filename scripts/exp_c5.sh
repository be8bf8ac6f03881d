# EXPERIMENT: config-5 bench, 8-step aligned graphs (default) against 4-step graphs, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c5
mkdir -p $O
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:>6} step {d['ms_per_step']*1e3:.1f} us  steps {d['steps']} warmup {d['warmup']}", flush=True)
PY
}
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload config5 --steps 32 --warmup 8 --no-cpu-baseline > $O/k8_$i.log 2>&1 || exit $?
  summ $O/k8_$i.log k8 || exit $?
  timeout -k 10 300 python bench.py --workload config5 --steps 32 --warmup 8 --steps-per-graph 4 --no-cpu-baseline > $O/k4_$i.log 2>&1 || exit $?
  summ $O/k4_$i.log k4 || exit $?
done
timeout -k 10 300 python bench.py --workload config5 --steps 30 --warmup 5 --no-cpu-baseline > $O/k8_30.log 2>&1 || exit $?
summ $O/k8_30.log k8_30
