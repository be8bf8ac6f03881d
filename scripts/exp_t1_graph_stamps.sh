# EXPERIMENT: T1 per-wave stamps inside the 8-step ring graph (GRAPH=1) vs eager, with and without
# the row gather (T1_ABLATE=32, timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for d in 0 32 16; do
  echo "== graph stamps, ablate $d"
  GRAPH=1 T1_ABLATE=$d timeout -k 10 200 python scripts/rows_stamps.py 2>&1 | grep -v amdgpu.ids || exit $?
done
echo "== eager stamps, ablate 0"
timeout -k 10 200 python scripts/rows_stamps.py 2>&1 | grep -v amdgpu.ids || exit $?
