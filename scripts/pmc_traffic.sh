# HBM traffic of the step's kernels from PMC counters (MI355X_MICROARCH.md "HBM" + "rocprofv3 PMC
# slots"): FETCH_SIZE and WRITE_SIZE in SEPARATE passes (they cannot share the 4 TCC slots), each
# pass a short bench run of its own under a hard time limit; summarised by scripts/pmc_summary.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit $?
ARGS="--steps 8 --warmup 0 --no-cpu-baseline --kernel-iters 4 ${BENCH_ARGS:-}"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/write -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/write.log 2>&1 || exit $?
python scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.json
cat gpurun_out/pmc/summary.json
