# Round 6: kernel trace of the world-1 sharded step (direct device-initiated exchange), and the
# bench lines for fine-grained vs coarse-grained receive buffers and the put form.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r06c}
mkdir -p gpurun_out/prof_$T
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o sh --output-format csv -- python3 bench.py --sharded --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/${T}_prof_sharded.log 2>&1 || exit $?
find gpurun_out/prof_$T -name "*kernel_stats*" | head -3
for m in fine-grained device; do
  TT_PEER_MEMORY=$m timeout -k 10 240 python bench.py --sharded --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/${T}_bench_sharded_$m.log 2>&1 || exit $?
  python -c "import json;l=[x for x in open('gpurun_out/${T}_bench_sharded_$m.log') if x.startswith('{')][-1];d=json.loads(l);print('$m',d['ms_per_step']*1e3,'us',d['config']['sharded']['exchange'])"
done
mkdir -p gpurun_out/prof_${T}_ov
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_ov -o sh --output-format csv -- python3 bench.py --sharded --overlap --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/${T}_prof_sharded_overlap.log 2>&1 || exit $?
find gpurun_out/prof_${T}_ov -name "*kernel_stats*" | head -3
