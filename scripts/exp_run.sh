set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
IDS=zipf timeout -k 10 200 python -u scripts/ring_stamps.py > gpurun_out/rs_zipf.log 2>&1 || exit $?
