# GPU: the DMP config-3 child over several seeds of its model init (tolerance margins per seed)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for s in 0 1 2 3 4 5; do
  TT_TEST_SEED=$s timeout -k 10 120 python tests/dmp_config3_check.py > gpurun_out/seed_$s.log 2>&1 || { echo "seed $s rc=$?"; tail -30 gpurun_out/seed_$s.log; exit 1; }
  grep MARGINS gpurun_out/seed_$s.log | sed "s/^/seed $s /"
done
