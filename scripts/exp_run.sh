set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/owner_update_stamps.py > gpurun_out/own.log 2>&1 || exit $?
