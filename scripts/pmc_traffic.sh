# PMC counters of the step's kernels (MI355X_MICROARCH.md "HBM" + "rocprofv3 PMC slots"), each pass a
# short bench run of its own under a hard time limit, summarised by scripts/pmc_summary.py:
#   fetch: FETCH_SIZE            (3 of the 4 TCC slots)
#   write: WRITE_SIZE            (2 TCC slots: cannot share a pass with FETCH_SIZE)
#   mfma:  SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES (SQ) + GRBM_GUI_ACTIVE (GRBM)
# BENCH_ARGS selects the workload (e.g. "--workload config5"); OUT names the summary directory.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit $?
ARGS="--steps 8 --warmup 0 --no-cpu-baseline --kernel-iters 4 ${BENCH_ARGS:-}"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/mfma -o run --output-format csv -- python3 bench.py $ARGS > $OUT/mfma.log 2>&1 || exit $?
python scripts/pmc_summary.py $OUT > $OUT/summary.json
cat $OUT/summary.json
