# Round 6: same-box A/B of a bench line between environment settings of the same library. VARS:
# space-separated variants, each NAME=VAL[,NAME=VAL...] ("-" for none), R interleaved rounds; prints
# ms per step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06h}_abenv
mkdir -p $O
for i in $(seq 1 ${R:-3}); do
  for v in ${VARS:-- TT_PEER_MERGED=0}; do
    n=$(echo "$v" | tr '=/,' '___')
    L=""
    [ "$v" != "-" ] && L=$(echo "$v" | tr ',' ' ')
    env $L timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-100} --warmup 20 ${BENCH_ARGS:---sharded} > $O/${n}_$i.log 2>&1 || exit $?
    python -c "
import json; d = json.loads([l for l in open('$O/${n}_$i.log') if l.startswith('{')][-1])
print('$v', round(d['ms_per_step'] * 1e3, 2), 'us', flush=True)" || exit $?
  done
done
