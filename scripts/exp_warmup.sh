# EXPERIMENT: the driver's 20-step line against the warm-up length (W = 5, the driver's, vs 40)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/warm
mkdir -p $O
for i in 1 2; do
  for w in 5 40 5; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup $w > $O/w${w}_$i.log 2>&1 || exit $?
    python - $O/w${w}_$i.log <<'PY' || exit $?
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"W {d['warmup']:>3} K {d['steps']} step {d['ms_per_step']*1e3:.2f} us", flush=True)
PY
  done
done
