set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_hf
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_hf -o hf --output-format csv -- python3 scripts/host_fed_probe.py > gpurun_out/prof_hf.log 2>&1 || exit $?
