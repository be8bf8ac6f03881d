# Round 6: one kernel trace (rocprofv3 --kernel-trace --stats) of a bench line; BENCH_ARGS picks it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r06j}
mkdir -p gpurun_out/prof_$T
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o tr --output-format csv -- python3 bench.py ${BENCH_ARGS:---sharded} --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/${T}_trace.log 2>&1 || exit $?
echo "trace ok"
