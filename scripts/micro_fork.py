"""EXPERIMENT: the cost of forking a captured HIP graph into parallel branches (torch streams +
events, as the multi-hot step does): a head kernel, then B branches of one kernel each, joined,
repeated; run under rocprofv3 --kernel-trace and read the gap between the head's end and each
branch kernel's start (scripts/timeline.py). B = 1 (a plain chain), 2, 4."""
import sys

import torch

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
x = [torch.zeros(1 << 22, device=dev) for _ in range(B + 1)]  # 16 MB each: ~5 us kernels
streams = [torch.cuda.Stream(device=dev) for _ in range(B)]
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream(device=dev)
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s):
        for step in range(4):
            x[0].mul_(1.0001)  # head
            ev = torch.cuda.Event()
            ev.record(s)
            for i in range(B):
                if i == 0:
                    x[1].add_(1.0)  # branch 0 stays on the capture stream
                else:
                    streams[i].wait_event(ev)
                    with torch.cuda.stream(streams[i]):
                        x[i + 1].add_(1.0)
            for i in range(1, B):
                s.wait_stream(streams[i])
torch.cuda.current_stream().wait_stream(s)
for _ in range(20):
    g.replay()
torch.cuda.synchronize()
print("done", B)
