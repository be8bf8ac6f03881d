# EXPERIMENT (timing only, wrong tail inputs): T1 without its dZ0 strip (128), its h strip (256), both
# (384), or every strip (896), against the same experiment library with all of them
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/strips
mkdir -p $O
for i in 1 2; do
  for d in 0 128 256 384 896; do
    TT_EXPERIMENT_LIB=1 TT_T1_DEBUG=$d timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 20 > $O/b_${d}_$i.log 2>&1 || exit $?
    python - $O/b_${d}_$i.log $d <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["roofline"]["kernels"]
print(f"skip={sys.argv[2]:>3} step {d['ms_per_step']*1e3:.2f} us  t1 {k['t1']['ms']*1e3:.2f}  tail {k['tail']['ms']*1e3:.2f}  t3 {k['t3']['ms']*1e3:.2f}", flush=True)
PY
  done
done
