set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/t1_wave_stamps.py > gpurun_out/t1w.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_q.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/t1_wave_stamps.py 4096 > gpurun_out/t1w_nt.log 2>&1 || exit $?
TT_T1_DEBUG=4096 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench_nt.log 2>&1 || exit $?
