"""Host-side costs of the host-fed pipeline's primitives on the GPU box (profiles/r03_h2d_probe.log):
issuing a pinned -> device copy of one group's columns (1.3 MB) on a side stream, waiting for an
event that already completed (synchronize vs a query spin), and a plain numpy -> pinned memcpy."""
import time

import numpy as np
import torch

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
n = 8 * 2 * 8192
pin = torch.zeros(n, dtype=torch.int64).pin_memory()
lab = torch.zeros(8 * 8192, dtype=torch.int32).pin_memory()
d = torch.zeros(n, dtype=torch.int64, device=dev)
dl = torch.zeros(8 * 8192, dtype=torch.int32, device=dev)
cs = torch.cuda.Stream(device=dev)
src = np.random.default_rng(0).integers(0, 1 << 30, n, dtype=np.int64)
for label, blocking in (("non_blocking", True), ("blocking", False)):
    ts = []
    for i in range(50):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(cs):
            d.copy_(pin, non_blocking=blocking)
            dl.copy_(lab, non_blocking=blocking)
            ev = torch.cuda.Event()
            ev.record(cs)
        ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    print(f"issue H2D ({label}): median {np.median(ts) * 1e6:.1f} us, min {min(ts) * 1e6:.1f} us")
ev = torch.cuda.Event()
ev.record(cs)
torch.cuda.synchronize()
ts = []
for i in range(50):
    t0 = time.perf_counter()
    ev.synchronize()
    ts.append(time.perf_counter() - t0)
print(f"synchronize() on a completed event: median {np.median(ts) * 1e6:.1f} us")
ts = []
for i in range(50):
    t0 = time.perf_counter()
    while not ev.query():
        pass
    ts.append(time.perf_counter() - t0)
print(f"query() on a completed event: median {np.median(ts) * 1e6:.1f} us")
pn = pin.numpy()
ts = []
for i in range(50):
    t0 = time.perf_counter()
    pn[:] = src
    ts.append(time.perf_counter() - t0)
print(f"numpy -> pinned memcpy 1 MB: median {np.median(ts) * 1e6:.1f} us")
# a pending copy: issue, then wait
ts, tq = [], []
for i in range(20):
    torch.cuda.synchronize()
    with torch.cuda.stream(cs):
        d.copy_(pin, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(cs)
    t0 = time.perf_counter()
    ev.synchronize()
    ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    with torch.cuda.stream(cs):
        d.copy_(pin, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(cs)
    t0 = time.perf_counter()
    while not ev.query():
        pass
    tq.append(time.perf_counter() - t0)
print(f"issue + wait for a 1 MB H2D: synchronize {np.median(ts) * 1e6:.1f} us, query spin {np.median(tq) * 1e6:.1f} us")
