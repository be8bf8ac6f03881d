"""Host-fed pipeline for the fused single-GPU step: TrainPipelineSparseDist's three stages
(03_model_training.py:618, :648) around ``FusedTwoTowerStep`` graphs.

The reference's loader yields host columns ``{user_id, product_id, label}`` (03:386-393) that
``transform_to_torchrec_batch`` turns into a KJT on the host, one element at a time (03:353-380).
Here the host only copies the raw columns; the transform (id 0 dropped, id % N) runs inside the
step's kernels. Per group of ``group`` batches (one HIP graph of ``group`` steps per device slot):

  stage 1  host     columns of group g+2 -> a pinned staging slot (CPU memcpy)
           copy     pinned slot -> device slot of group g+2 (async H2D on the copy stream), after
                    the graph that last read that device slot has finished (event)
  stage 2  copy     the device slot of group g+1 is complete (its H2D event) — the single-hot
                    step has no separate input_dist: the KJT build is fused into T1
  stage 3  compute  graph replay of group g on the step's stream, after its H2D event

``depth`` device / pinned slots rotate (4: one computing, one landed for the next group, one being
filled, one whose graph may still be draining); the host fills group g+2 right after queuing group
g's graph, into the slot of group g-2. The host waits for that slot's last graph itself (an event it
almost never has to wait for) and then issues the H2D with no device-side dependency: on this ROCm
stack a hipMemcpyAsync queued behind a cross-stream event wait blocked the calling thread until the
event fired (measured: 222 us of host time per group for the 1 MB id copy, 0.5 ms per group in all,
against 0.29 ms of device work; profiles/r03_bench_hostfed*.log), so the host never ran ahead.

With ``ring`` (the default when the step supports it) the graphs are the PRODUCTION ring's
(``FusedTwoTowerStep.capture_ring`` over the slots' batches: each step files the next batch's dedup
table, rows looked up once are updated inside T1): group g's graph also reads the first batch of
group g+1 (its last step files that batch), so group g starts after BOTH slots have landed; the
first batch's table is primed when a run starts. ``trace`` records host timestamps per group
(host copy, H2D issue, waits, replay issue) and device events around every replay, for
``summary()``.
"""
from __future__ import annotations

from typing import Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib


class HostFedPipeline:
    def __init__(self, step, group: int = 8, depth: int = 4, ring: Optional[bool] = None, trace: bool = False):
        """step: a FusedTwoTowerStep (single-hot columns). group: batches per graph replay."""
        if getattr(step, "kjt_input", False):
            raise _lib.TTError("HostFedPipeline: single-hot column input only")
        self.step = step
        self.group = int(group)
        self.depth = int(depth)
        self.ring = step.ring_supported() if ring is None else bool(ring)
        if self.group < 1 or self.depth < 4:
            raise _lib.TTError("HostFedPipeline: group >= 1, depth >= 4")
        self.trace = [] if trace else None
        dev, B, F = step.device, step.B, step.F
        self.device = dev
        idt = step.id_dtype
        # device slots: per slot, `group` batches of F id columns + labels (read in place by graphs)
        self.dev_ids = [torch.zeros(self.group, F, B, dtype=idt, device=dev) for _ in range(self.depth)]
        self.dev_lab = [torch.zeros(self.group, B, dtype=torch.int32, device=dev) for _ in range(self.depth)]
        self.pin_ids = [torch.zeros(self.group, F, B, dtype=idt).pin_memory() for _ in range(self.depth)]
        self.pin_lab = [torch.zeros(self.group, B, dtype=torch.int32).pin_memory() for _ in range(self.depth)]
        # numpy views of the pinned slots: the host copy is a plain memcpy per column
        self.pin_ids_np = [t.numpy() for t in self.pin_ids]
        self.pin_lab_np = [t.numpy() for t in self.pin_lab]
        self.copy_stream = torch.cuda.Stream(device=dev)
        self.h2d_done: List[Optional[torch.cuda.Event]] = [None] * self.depth   # slot landed
        self.slot_free: List[Optional[torch.cuda.Event]] = [None] * self.depth  # graph that read it ended
        self.filled: List[int] = [0] * self.depth                               # batches in the slot
        # one graph per slot (group steps, or fewer for a final partial group: eager steps)
        batches = []
        for s in range(self.depth):
            for j in range(self.group):
                batches.append(([self.dev_ids[s][j, f] for f in range(F)], self.dev_lab[s][j]))
        self._batches = batches
        if self.ring:
            if (self.depth * self.group) % 2:
                raise _lib.TTError("HostFedPipeline: the ring needs an even number of slot batches")
            step.capture_ring(batches, steps_per_graph=self.group)
            self.graphs = list(step.ring_graphs)
            assert step.ring_offset == 0
        else:
            step.capture_pool(batches, steps_per_graph=self.group)
            self.graphs = list(step.pool_graphs)

    # -- stage 1
    def _t(self):
        import time

        return time.perf_counter()

    def _fill(self, slot: int, it: Iterator) -> int:
        """Host columns of up to `group` batches -> pinned slot -> async H2D. Returns the count."""
        t0 = self._t() if self.trace is not None else 0.0
        if self.h2d_done[slot] is not None:
            self.h2d_done[slot].synchronize()  # the pinned buffer's previous copy has left
        t1 = self._t() if self.trace is not None else 0.0
        n = 0
        for j in range(self.group):
            try:
                cols, labels = next(it)
            except StopIteration:
                break
            for f, c in enumerate(cols):
                self.pin_ids_np[slot][j, f] = np.asarray(c)
            self.pin_lab_np[slot][j] = np.asarray(labels)
            n += 1
        self.filled[slot] = n
        t2 = self._t() if self.trace is not None else 0.0
        if n == 0:
            return 0
        tr = self.trace is not None
        if self.slot_free[slot] is not None:
            self.slot_free[slot].synchronize()  # the graph that last read this slot (two groups back)
        with torch.cuda.stream(self.copy_stream):
            t3 = self._t() if tr else 0.0
            self.dev_ids[slot][:n].copy_(self.pin_ids[slot][:n], non_blocking=True)
            t4 = self._t() if tr else 0.0
            self.dev_lab[slot][:n].copy_(self.pin_lab[slot][:n], non_blocking=True)
            t5 = self._t() if tr else 0.0
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
        self.h2d_done[slot] = ev
        if tr:
            self.trace.append(("fill", slot, n, t0, t1, t2, self._t(), (t3, t4, t5)))
        return n

    # -- stage 3
    def _compute(self, slot: int) -> None:
        t0 = self._t() if self.trace is not None else 0.0
        main = torch.cuda.current_stream(self.device)
        main.wait_event(self.h2d_done[slot])
        nxt = (slot + 1) % self.depth
        if self.ring and self.filled[nxt] and self.h2d_done[nxt] is not None:
            main.wait_event(self.h2d_done[nxt])  # the ring's last step files group g+1's first batch
        n = self.filled[slot]
        if self.trace is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(main)
        t1 = self._t() if self.trace is not None else 0.0
        if n == self.group:
            self.graphs[slot].replay()
        elif self.ring:  # a final partial group: the production steps, eagerly
            st, nb = self.step, len(self._batches)
            for j in range(n):
                i = slot * self.group + j
                cols, lab = self._batches[i]
                st.ring_step(cols, lab, i % 2, self._batches[(i + 1) % nb][0])
        else:  # a final partial group: the same kernels, eagerly
            st = self.step
            keep = st.cols, st.labels
            try:
                for j in range(n):
                    st.cols = [self.dev_ids[slot][j, f] for f in range(st.F)]
                    st.labels = self.dev_lab[slot][j]
                    st.step()
            finally:
                st.cols, st.labels = keep
        ev = torch.cuda.Event(enable_timing=self.trace is not None)
        ev.record(main)
        self.slot_free[slot] = ev
        if self.trace is not None:
            self.trace.append(("compute", slot, n, t0, t1, self._t(), (e0, ev)))

    def summary(self) -> dict:
        """From ``trace``: mean host milliseconds per group in each stage (fill: the wait for the
        pinned slot's previous copy, the host memcpy, the H2D issue; compute: the wait / replay
        issue) and the device milliseconds per group between the replay's start and end events, and
        the host's total per group (the loop's period)."""
        if not self.trace:
            return {}
        torch.cuda.synchronize(self.device)
        fills = [e for e in self.trace if e[0] == "fill"]
        comps = [e for e in self.trace if e[0] == "compute"]
        ms = lambda a, b: (b - a) * 1e3  # noqa: E731
        out = {
            "groups": len(comps),
            "host_ms_fill_wait_prev_copy": sum(ms(e[3], e[4]) for e in fills) / max(1, len(fills)),
            "host_ms_fill_memcpy": sum(ms(e[4], e[5]) for e in fills) / max(1, len(fills)),
            "host_ms_fill_h2d_issue": sum(ms(e[5], e[6]) for e in fills) / max(1, len(fills)),
            "host_ms_fill_wait_event": sum(ms(e[5], e[7][0]) for e in fills) / max(1, len(fills)),
            "host_ms_fill_copy_ids": sum(ms(e[7][0], e[7][1]) for e in fills) / max(1, len(fills)),
            "host_ms_fill_copy_labels": sum(ms(e[7][1], e[7][2]) for e in fills) / max(1, len(fills)),
            "host_ms_fill_record": sum(ms(e[7][2], e[6]) for e in fills) / max(1, len(fills)),
            "host_ms_compute_issue": sum(ms(e[3], e[5]) for e in comps) / max(1, len(comps)),
            "device_ms_per_group": sum(e[6][0].elapsed_time(e[6][1]) for e in comps) / max(1, len(comps)),
        }
        if len(comps) > 1:
            out["host_ms_period"] = ms(comps[0][3], comps[-1][3]) / (len(comps) - 1)
        return out

    def run(self, host_batches: Iterable[Tuple[Sequence, object]], max_steps: Optional[int] = None) -> int:
        """Train on host batches ((id columns, labels) per batch: numpy arrays or CPU tensors of the
        step's id dtype / int) until the iterable (or max_steps) is exhausted; returns the steps
        run. Asynchronous: synchronize the device before reading results."""
        it = iter(host_batches)
        if max_steps is not None:
            import itertools

            it = itertools.islice(it, max_steps)
        D = self.depth
        steps = 0
        for k in range(D):  # a previous run's slots are refilled from group 0
            self.filled[k] = 0
        # prologue: groups 0 and 1 in flight
        for g in range(2):
            self._fill(g % D, it)
        if self.ring and self.filled[0]:
            # the first batch's dedup table, once its slot has landed (every later table is filed
            # by the step before its batch); tables left over from a previous run are emptied
            main = torch.cuda.current_stream(self.device)
            main.wait_event(self.h2d_done[0])
            self.step.ring_reset()
            self.step.ring_prime(self._batches[0][0], 0)
        g = 0
        while True:
            slot = g % D
            if self.filled[slot] == 0:
                break
            self._compute(slot)
            steps += self.filled[slot]
            self._fill((g + 2) % D, it)  # the slot of group g - 2
            g += 1
        return steps


def synthetic_host_batches(num_embeddings: Sequence[int], B: int, n: int, seed: int = 0, zero_frac: float = 0.0):
    """n host batches of single-hot id columns (int64, uniform over [0, N)) and Bernoulli labels —
    what the reference's dataloader yields per batch (03:386-393), as numpy arrays."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        cols = []
        for N in num_embeddings:
            c = rng.integers(0, N, B, dtype=np.int64)
            if zero_frac:
                c[rng.random(B) < zero_frac] = 0
            cols.append(c)
        out.append((cols, rng.integers(0, 2, B, dtype=np.int32)))
    return out
