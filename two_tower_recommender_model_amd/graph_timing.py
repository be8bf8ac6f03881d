"""Per-launch device time INSIDE a replayed HIP graph, with HIP events (bench instrumentation).

torch refuses external (graph-node) events on ROCm, so this edits the captured graph directly:
capture with ``torch.cuda.CUDAGraph(keep_graph=True)``, then for each kernel node of the linear
launch chain insert an event-record node before and after it (hipGraphAddEventRecordNode + edge
rewiring), instantiate, replay, and read hipEventElapsedTime per pair. The events are recorded on
the stream the graph (and so each kernel) runs on.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Tuple

_hip = None


def _lib():
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
        vp, sz = C.c_void_p, C.c_size_t
        _hip.hipGraphGetRootNodes.argtypes = [vp, C.POINTER(vp), C.POINTER(sz)]
        _hip.hipGraphNodeGetDependentNodes.argtypes = [vp, C.POINTER(vp), C.POINTER(sz)]
        _hip.hipGraphNodeGetType.argtypes = [vp, C.POINTER(C.c_int)]
        _hip.hipEventCreate.argtypes = [C.POINTER(vp)]
        _hip.hipEventDestroy.argtypes = [vp]
        _hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), vp, vp]
        _hip.hipGraphAddEventRecordNode.argtypes = [C.POINTER(vp), vp, C.POINTER(vp), sz, vp]
        _hip.hipGraphAddDependencies.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), sz]
        _hip.hipGraphRemoveDependencies.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), sz]
    return _hip


def _ok(rc, what):
    if rc != 0:
        _lib().hipGetLastError()  # do not leave the error for the next launch check to find
        raise RuntimeError(f"{what}: hipError {rc}")


def _dependents(node) -> List[int]:
    h = _lib()
    n = C.c_size_t(0)
    _ok(h.hipGraphNodeGetDependentNodes(node, None, C.byref(n)), "hipGraphNodeGetDependentNodes")
    arr = (C.c_void_p * max(1, n.value))()
    _ok(h.hipGraphNodeGetDependentNodes(node, arr, C.byref(n)), "hipGraphNodeGetDependentNodes")
    return [arr[i] for i in range(n.value)]


def linear_kernel_chain(raw_graph: int) -> Optional[List[int]]:
    """The graph's nodes in dependency order if they form one chain (one stream), else None."""
    h = _lib()
    n = C.c_size_t(0)
    _ok(h.hipGraphGetRootNodes(C.c_void_p(raw_graph), None, C.byref(n)), "hipGraphGetRootNodes")
    if n.value != 1:
        return None
    arr = (C.c_void_p * 1)()
    _ok(h.hipGraphGetRootNodes(C.c_void_p(raw_graph), arr, C.byref(n)), "hipGraphGetRootNodes")
    chain = [arr[0]]
    while True:
        d = _dependents(chain[-1])
        if not d:
            return chain
        if len(d) != 1:
            return None
        chain.append(d[0])


class GraphLaunchTimer:
    """Event pairs around the kernel nodes ``which`` (indices into the chain's kernel nodes) of a
    keep_graph capture. Call ``elapsed()`` after each replay + synchronize."""

    def __init__(self, graph, which: List[int]):
        h = _lib()
        raw = C.c_void_p(graph.raw_cuda_graph())
        chain = linear_kernel_chain(raw.value)
        if chain is None:
            raise RuntimeError("graph is not a single launch chain")
        kernels = []
        for node in chain:
            t = C.c_int(-1)
            _ok(h.hipGraphNodeGetType(node, C.byref(t)), "hipGraphNodeGetType")
            if t.value == 0:  # hipGraphNodeTypeKernel
                kernels.append(node)
        pos = {n: i for i, n in enumerate(chain)}
        pred = {}  # a node's current predecessor once an event node was put in front of it
        self.pairs: List[Tuple[C.c_void_p, C.c_void_p]] = []
        for k in which:
            node = kernels[k]
            i = pos[node]
            prev = pred.get(node, chain[i - 1] if i > 0 else None)
            nxt = chain[i + 1] if i + 1 < len(chain) else None
            ev0, ev1 = C.c_void_p(), C.c_void_p()
            _ok(h.hipEventCreate(C.byref(ev0)), "hipEventCreate")
            _ok(h.hipEventCreate(C.byref(ev1)), "hipEventCreate")
            n0, n1 = C.c_void_p(), C.c_void_p()
            one = lambda x: (C.c_void_p * 1)(x)  # noqa: E731
            if prev is not None:
                _ok(h.hipGraphRemoveDependencies(raw, one(prev), one(node), 1), "hipGraphRemoveDependencies")
                _ok(h.hipGraphAddEventRecordNode(C.byref(n0), raw, one(prev), 1, ev0), "hipGraphAddEventRecordNode")
            else:
                _ok(h.hipGraphAddEventRecordNode(C.byref(n0), raw, None, 0, ev0), "hipGraphAddEventRecordNode")
            _ok(h.hipGraphAddDependencies(raw, one(n0), one(node), 1), "hipGraphAddDependencies")
            if nxt is not None:
                _ok(h.hipGraphRemoveDependencies(raw, one(node), one(nxt), 1), "hipGraphRemoveDependencies")
            _ok(h.hipGraphAddEventRecordNode(C.byref(n1), raw, one(node), 1, ev1), "hipGraphAddEventRecordNode")
            if nxt is not None:
                _ok(h.hipGraphAddDependencies(raw, one(n1), one(nxt), 1), "hipGraphAddDependencies")
                pred[nxt] = n1.value
            self.pairs.append((ev0, ev1))
        graph.instantiate()

    def elapsed(self) -> List[float]:
        """ms of each instrumented launch in the last replay (call after synchronize)."""
        h = _lib()
        out = []
        for a, b in self.pairs:
            ms = C.c_float(0.0)
            _ok(h.hipEventElapsedTime(C.byref(ms), a, b), "hipEventElapsedTime")
            out.append(ms.value)
        return out

    def close(self) -> None:
        h = _lib()
        for a, b in self.pairs:
            h.hipEventDestroy(a)
            h.hipEventDestroy(b)
        self.pairs = []
