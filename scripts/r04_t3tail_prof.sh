#!/bin/bash
# kernel durations of the ring with T3 in the tail vs the three-launch ring
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/t3t_off -o run -- python3 bench.py --steps 100 --warmup 20 > gpurun_out/t3t_prof_off.log 2>&1 && \
TT_T3_IN_TAIL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/t3t_on -o run -- python3 bench.py --steps 100 --warmup 20 > gpurun_out/t3t_prof_on.log 2>&1 || exit 1
for d in t3t_off t3t_on; do f=$(find gpurun_out/$d -name '*kernel_stats.csv' | head -1); echo "== $d"; python3 - "$f" <<'PY'
import csv,sys
r=list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x:-float(x['TotalDurationNs']))
for x in r[:8]: print(x['Calls'], round(float(x['AverageNs'])/1000,2), x['Name'][:110])
PY
done
