"""Per-step timeline from a rocprofv3 kernel-trace CSV: every dispatch's start / end relative to the
start of the step's anchor kernel (first dispatch of a name containing argv[2]), median over the
steps after the first argv[3] (default 10) anchors. Shows what overlaps what inside a graph step."""
import csv, statistics, sys
from collections import OrderedDict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2]
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 10
steps, cur = [], None
for r in rows:
    name = r["Kernel_Name"]
    if anchor in name:
        cur = []
        steps.append(cur)
    if cur is not None:
        cur.append((name[:48], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
steps = steps[skip:-1]
acc = OrderedDict()
for st in steps:
    t0 = st[0][1]
    seen = {}
    for name, s, e in st:
        k = (name, seen.get(name, 0))
        seen[name] = seen.get(name, 0) + 1
        acc.setdefault(k, []).append(((s - t0) / 1e3, (e - t0) / 1e3))
span = [(st[-1][2] - st[0][1]) / 1e3 for st in steps]
nxt = [(steps[i + 1][0][1] - steps[i][0][1]) / 1e3 for i in range(len(steps) - 1)]
print(f"steps {len(steps)}  anchor-to-anchor {statistics.median(nxt) if nxt else 0:.1f} us  "
      f"first-start-to-last-end {statistics.median(span):.1f} us")
for (name, i), v in acc.items():
    if len(v) < len(steps) // 2:
        continue
    s = statistics.median(a for a, _ in v)
    e = statistics.median(b for _, b in v)
    print(f"{s:8.1f} {e:8.1f} {e - s:8.1f}  {name}#{i}")
