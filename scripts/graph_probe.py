"""EXPERIMENT: what a captured fork looks like inside the HIP graph (node types, edges) — the
micro_fork.py graph with B branches, keep_graph=True, read through hipGraphGetNodes / GetEdges."""
import ctypes as C
import sys

import torch

hip = C.CDLL("libamdhip64.so", mode=C.RTLD_GLOBAL)
dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
x = [torch.zeros(1 << 22, device=dev) for _ in range(B + 1)]
streams = [torch.cuda.Stream(device=dev) for _ in range(B)]
g = torch.cuda.CUDAGraph(keep_graph=True)
s = torch.cuda.Stream(device=dev)
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s):
        x[0].mul_(1.0001)
        ev = torch.cuda.Event()
        ev.record(s)
        for i in range(B):
            if i == 0:
                x[1].add_(1.0)
            else:
                streams[i].wait_event(ev)
                with torch.cuda.stream(streams[i]):
                    x[i + 1].add_(1.0)
        for i in range(1, B):
            s.wait_stream(streams[i])
        x[0].mul_(1.0001)
graph = C.c_void_p(g.raw_cuda_graph())
n = C.c_size_t(0)
hip.hipGraphGetNodes(graph, None, C.byref(n))
nodes = (C.c_void_p * n.value)()
hip.hipGraphGetNodes(graph, nodes, C.byref(n))
names = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty", 6: "waitEvent", 7: "eventRecord"}
idx = {nodes[i]: i for i in range(n.value)}
for i in range(n.value):
    t = C.c_int(0)
    hip.hipGraphNodeGetType(C.c_void_p(nodes[i]), C.byref(t))
    nd = C.c_size_t(0)
    hip.hipGraphNodeGetDependencies(C.c_void_p(nodes[i]), None, C.byref(nd))
    deps = (C.c_void_p * max(1, nd.value))()
    hip.hipGraphNodeGetDependencies(C.c_void_p(nodes[i]), deps, C.byref(nd))
    print(i, names.get(t.value, t.value), "deps", [idx.get(deps[k]) for k in range(nd.value)])
