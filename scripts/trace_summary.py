"""Median device time per (kernel, grid, workgroup) from a rocprofv3 kernel-trace CSV, in dispatch order."""
import csv, statistics, sys
from collections import OrderedDict
d = OrderedDict()
for r in csv.DictReader(open(sys.argv[1])):
    k = (r["Kernel_Name"][:40], r["Grid_Size_X"], r["Workgroup_Size_X"])
    d.setdefault(k, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in d.items():
    print(k, len(v), statistics.median(v))
