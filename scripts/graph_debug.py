import os, sys, ctypes as C
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep
from two_tower_recommender_model_amd import graph_timing as gt
dev = torch.device("cuda:0")
N = [100000, 200000]; B = 1024
st = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, dev)
g = torch.Generator(device=dev).manual_seed(1)
batches = [([torch.randint(0, n, (B,), generator=g, device=dev) for n in N], torch.randint(0, 2, (B,), generator=g, device=dev, dtype=torch.int32)) for _ in range(2)]
st.capture_pool(batches, steps_per_graph=2, keep_graph=True)
graph = st.pool_graphs[0]
h = gt._lib()
raw = C.c_void_p(graph.raw_cuda_graph())
n = C.c_size_t(0)
print("roots rc", h.hipGraphGetRootNodes(raw, None, C.byref(n)), n.value)
arr = (C.c_void_p * max(1, n.value))()
h.hipGraphGetRootNodes(raw, arr, C.byref(n))
seen = []
frontier = [arr[i] for i in range(n.value)]
while frontier:
    node = frontier.pop(0)
    t = C.c_int(-1); h.hipGraphNodeGetType(node, C.byref(t))
    d = gt._dependents(node)
    print("node", node, "type", t.value, "deps", len(d))
    seen.append(node)
    frontier += [x for x in d if x not in seen and x not in frontier]
h.hipGraphRemoveDependencies.restype = C.c_int
chain = gt.linear_kernel_chain(raw.value)
print("chain", chain is not None and len(chain))
one = lambda x: (C.c_void_p * 1)(x)
rc = h.hipGraphRemoveDependencies(raw, one(chain[0]), one(chain[1]), 1)
print("remove rc", rc)
