# EXPERIMENT: what T1's prologue costs — the ring step and T1 with the weight-image fill and/or the
# row gather skipped (experiment library; timing only, wrong results), then per-wave stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/exp_t1p
mkdir -p $O
for d in 0 16 32 48 0; do
  TT_EXPERIMENT_LIB=1 TT_T1_DEBUG=$d timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 20 > $O/bench_$d.log 2>&1 || exit $?
  python - $O/bench_$d.log $d <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["roofline"]["kernels"]
print(f"ablate={sys.argv[2]:>2} step {d['ms_per_step']*1e3:.2f} us  t1 {k['t1']['ms']*1e3:.2f}  tail {k['tail']['ms']*1e3:.2f}  t3 {k['t3']['ms']*1e3:.2f}")
PY
done
for d in 0 16 32; do
  echo "== stamps, ablate $d"
  T1_ABLATE=$d timeout -k 10 200 python scripts/rows_stamps.py || exit $?
done
