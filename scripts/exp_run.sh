set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export TT_EXPERIMENT_LIB=1
timeout -k 10 200 python3 scripts/ring_stamps.py > gpurun_out/ring_stamps_u.log 2>&1 || exit $?
IDS=zipf timeout -k 10 200 python3 scripts/ring_stamps.py > gpurun_out/ring_stamps_z.log 2>&1 || exit $?
timeout -k 10 200 python3 scripts/t2_stamps.py > gpurun_out/t2_stamps.log 2>&1 || exit $?
