set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for b in 1 2 4; do
  mkdir -p gpurun_out/fork$b
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/fork$b -o f --output-format csv -- python3 scripts/micro_fork.py $b > gpurun_out/fork$b.log 2>&1 || exit 1
  python3 - $b <<'PY'
import csv, sys, statistics as S
b = sys.argv[1]
rows = sorted(csv.DictReader(open(f"gpurun_out/fork{b}/f_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "mul" in r["Kernel_Name"] or "add" in r["Kernel_Name"] or "Mul" in r["Kernel_Name"] or "Add" in r["Kernel_Name"]]
gaps, heads = [], []
for i, r in enumerate(rows):
    if "MulFunctor" in r["Kernel_Name"] or "mul" in r["Kernel_Name"].lower() and "add" not in r["Kernel_Name"].lower():
        end = int(r["End_Timestamp"])
        nxt = [int(q["Start_Timestamp"]) - end for q in rows[i + 1:i + 1 + int(b)]]
        gaps.append(nxt)
        heads.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
g = [sorted(x) for x in gaps[5:]]
print(f"B={b}: head {S.median(heads):.1f} us; branch starts after the head's end (us, median over forks):",
      [round(S.median([x[k] for x in g if len(x) > k]) / 1e3, 1) for k in range(int(b))])
PY
done
