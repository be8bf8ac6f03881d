"""Mean per-dispatch value of every counter of a rocprofv3 --pmc run, per tt:: kernel.

    python scripts/pmc_dump.py gpurun_out/pmc_x     # the -d directory of one pass
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    acc = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "tt::" not in name:
                continue
            k = name.split("(")[0].replace("void ", "")
            did = r.get("Dispatch_Id") or r.get("Correlation_Id")
            c = r["Counter_Name"]
            acc[k][c][did] = acc[k][c].get(did, 0.0) + float(r["Counter_Value"])
    for k in sorted(acc):
        print(k)
        for c in sorted(acc[k]):
            v = list(acc[k][c].values())
            print(f"  {c:32s} {sum(v) / len(v):16.1f}  ({len(v)} dispatches)")


if __name__ == "__main__":
    main(sys.argv[1])
