# round 4 evidence: PMC passes (north star), the default bench line (with the CPU baseline), its
# kernel trace, and the other workloads' lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc_r04c bash scripts/pmc_traffic.sh > gpurun_out/pmc_r04c.log 2>&1 || { tail -20 gpurun_out/pmc_r04c.log; exit 1; }
cp gpurun_out/pmc_r04c/summary.json profiles/r04c_pmc_traffic.json
timeout -k 10 400 python bench.py > gpurun_out/r04c_bench.log 2>&1 || { tail -20 gpurun_out/r04c_bench.log; exit 1; }
tail -1 gpurun_out/r04c_bench.log | cut -c1-400
mkdir -p gpurun_out/prof_r04c
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04c -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/r04c_bench_prof.log 2>&1 || exit 1
for w in "--workload config2" "--ids zipf" "--workload config5" "--path dropin" "--sharded"; do
  n=$(echo "$w" | tr -d ' -')
  timeout -k 10 400 python bench.py $w --no-cpu-baseline > gpurun_out/r04c_bench_$n.log 2>&1 || { tail -5 gpurun_out/r04c_bench_$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04c_bench_$n.log) $(grep -o '"value": [0-9.]*' gpurun_out/r04c_bench_$n.log | head -1)"
done
