"""Per-launch PMC figures of each tt:: kernel from the passes of scripts/pmc_traffic.sh.

HBM bytes: FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB. gfx950 correction
(MI355X_MICROARCH.md, HBM): FETCH_SIZE reports 1/2 of the bytes of wide (16 B/lane) coalesced reads,
so read bytes = 2 x FETCH_SIZE x 1024 (every tt:: kernel reads its rows as 16-B vectors);
WRITE_SIZE is exact for 16-B-per-lane stores: write bytes = WRITE_SIZE x 1024.

MFMA (the mfma pass): flops = SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 (rocprofv3's MfmaFlopsBF16);
utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (kernel cycles x 1024 SIMDs), kernel cycles =
GRBM_GUI_ACTIVE / 8 (rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs: MI355X_MICROARCH.md, DVFS
give-back) — rocprofv3's MfmaUtil expression with that per-XCD reading.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 1024


def load(d, counter):
    """{kernel: [per-dispatch values]} (values of one dispatch summed over its rows)."""
    acc = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"]
            if "tt::" not in name:
                continue
            k = name.split("(")[0].replace("void ", "")
            did = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(len(acc[k]))
            acc[k][did] = acc[k].get(did, 0.0) + float(r["Counter_Value"])
    return {k: list(v.values()) for k, v in acc.items()}


def mean(v):
    return sum(v) / len(v) if v else None


def main(root):
    fetch = load(os.path.join(root, "fetch"), "FETCH_SIZE")
    write = load(os.path.join(root, "write"), "WRITE_SIZE")
    mops = load(os.path.join(root, "mfma"), "SQ_INSTS_VALU_MFMA_MOPS_BF16")
    busy = load(os.path.join(root, "mfma"), "SQ_VALU_MFMA_BUSY_CYCLES")
    grbm = load(os.path.join(root, "mfma"), "GRBM_GUI_ACTIVE")
    out = {}
    for k in sorted(set(fetch) | set(write) | set(mops)):
        f, w = fetch.get(k, []), write.get(k, [])
        rd = 2.0 * 1024.0 * mean(f) if f else None
        wr = 1024.0 * mean(w) if w else None
        e = {"launches": [len(f), len(w)], "read_bytes": rd, "write_bytes": wr, "hbm_bytes": (rd or 0.0) + (wr or 0.0)}
        if mops.get(k):
            fl, bc, gc = mean(mops[k]) * 512.0, mean(busy.get(k, [])), mean(grbm.get(k, []))
            e["mfma_bf16_flop"] = fl
            e["mfma_busy_cycles"] = bc
            e["grbm_gui_active"] = gc
            if bc is not None and gc:
                e["mfma_util"] = bc / (gc / 8.0 * SIMDS)
                e["clock_cycles"] = gc / 8.0
        out[k] = e
    json.dump({"correction": "read = 2 x FETCH_SIZE KiB (gfx950 wide reads), write = WRITE_SIZE KiB; "
                             "mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)",
               "kernels": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
