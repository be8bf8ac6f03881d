set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_multiproc_rehearsal.py tests/test_gpu_sharded.py > gpurun_out/t_reh.log 2>&1 || exit $?
