# graph fork / join cost under HIP runtime graph-queue settings
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {  # $1 tag, $2 B, env from the caller
  mkdir -p gpurun_out/fk_$1
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/fk_$1 -o f --output-format csv -- python3 scripts/micro_fork.py $2 > gpurun_out/fk_$1.log 2>&1 || return 1
  python3 - gpurun_out/fk_$1/f_kernel_trace.csv $2 $1 <<'PY'
import csv, sys, statistics as S
path, b, tag = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "elementwise" in r["Kernel_Name"] or "Functor" in r["Kernel_Name"]]
heads = [k for k, r in enumerate(rows) if "Mul" in r["Kernel_Name"]]
fk, jn, ov = [], [], []
for h1, h2 in zip(heads, heads[1:]):
    br = rows[h1 + 1:h2]
    if len(br) != b:
        continue
    he = int(rows[h1]["End_Timestamp"])
    st = sorted(int(r["Start_Timestamp"]) - he for r in br)
    fk.append(st)
    jn.append(int(rows[h2]["Start_Timestamp"]) - max(int(r["End_Timestamp"]) for r in br))
    ov.append(max(int(r["End_Timestamp"]) for r in br) - min(int(r["Start_Timestamp"]) for r in br))
fk = fk[3:]
print(f"{tag} B={b}: fork starts {[round(S.median([x[k] for x in fk]) / 1e3, 1) for k in range(b)]} us, "
      f"join {S.median(jn[3:]) / 1e3:.1f} us, branch span {S.median(ov[3:]) / 1e3:.1f} us")
PY
}
run base4 4 && DEBUG_HIP_FORCE_GRAPH_QUEUES=1 run q1_4 4 && DEBUG_HIP_FORCE_GRAPH_QUEUES=2 run q2_4 4 && DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 run nopc4 4 && DEBUG_HIP_FORCE_GRAPH_QUEUES=1 run q1_2 2
