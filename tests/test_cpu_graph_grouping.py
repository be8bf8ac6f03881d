"""Host logic of the multi-step graph grouping (no GPU): which captured graphs a run replays.

FusedTwoTowerStep.run / replay_pool walk the cursor through the resident pool and replay k-step
graphs where the grouping offset allows, aligned smaller graphs (k/2, ..., 2) and single-step graphs
otherwise; align_ring / align_pool move the grouping so that a run of n steps after w others replays
its remainder first and then only k-step graphs. Checked here on stand-in objects whose graphs record
their replays (the real graphs are HIP graphs: tests/test_gpu_multihot.py, tests/test_gpu_ring.py)."""
import types

import pytest

from two_tower_recommender_model_amd.fused import FusedTwoTowerStep


class _G:
    def __init__(self, log, name, steps):
        self.log, self.name, self.steps = log, name, steps

    def replay(self):
        self.log.append((self.name, self.steps))


def _pool(n, k, offset):
    """A stand-in multi-hot pool of n batches grouped from ``offset`` (graphs as in _kjt_groups)."""
    log = []
    o = types.SimpleNamespace(pool_cursor=0, steps_per_graph=k, pool_offset=offset, log=log)
    span = lambda j, sz: [(offset + j + t) % n for t in range(sz)]  # noqa: E731
    o.pool_graphs = [_G(log, f"s{i}", [i]) for i in range(n)]
    o.pool_graphs_k = [_G(log, f"k{j}", span(j, k)) for j in range(0, n, k)]
    o.pool_mid, sz = {}, k // 2
    while sz >= 2:
        o.pool_mid[sz] = [_G(log, f"m{sz}_{j}", span(j, sz)) for j in range(0, n, sz)]
        sz //= 2

    def regroup(off):
        fresh = _pool(n, k, off)
        for a in ("pool_graphs", "pool_graphs_k", "pool_mid", "pool_offset"):
            setattr(o, a, getattr(fresh, a))
        for g in o.pool_graphs + o.pool_graphs_k + [g for v in o.pool_mid.values() for g in v]:
            g.log = log

    o._kjt_groups = regroup
    return o


def _steps(log):
    return [s for _, steps in log for s in steps]


@pytest.mark.parametrize("n,k,w,K", [(8, 8, 5, 20), (8, 4, 1, 6), (16, 8, 10, 50), (4, 2, 3, 7), (8, 8, 0, 16)])
def test_pool_run_is_consecutive_and_timed_region_uses_big_graphs(n, k, w, K):
    o = _pool(n, k, 0)
    FusedTwoTowerStep.align_pool(o, K, after=w)
    FusedTwoTowerStep.replay_pool(o, w)
    warm = list(o.log)
    o.log.clear()
    FusedTwoTowerStep.replay_pool(o, K)
    timed = list(o.log)
    # every step exactly once, in pool order, continuing at the cursor
    assert _steps(warm) + _steps(timed) == [i % n for i in range(w + K)]
    assert o.pool_cursor == (w + K) % n
    # the timed region: the remainder first (no single-step graph when it is a sum of the captured
    # sizes), then only k-step graphs
    sizes = [len(steps) for _, steps in timed]
    rem = K % k
    assert sum(sizes) == K and sizes[len(sizes) - K // k:] == [k] * (K // k)
    head = sizes[:len(sizes) - K // k]
    assert sum(head) == rem and all(s > 1 for s in head) == (rem % 2 == 0 or k == 1)


def test_ring_run_matches_pool_grouping():
    """The single-hot ring's run() follows the same rule (its graphs in ring_graphs / ring_mid /
    ring_small, grouping offset ring_offset)."""
    n, k = 16, 8
    log = []
    o = types.SimpleNamespace(ring_cursor=0, ring_k=k, ring_offset=3)
    span = lambda j, sz: [(3 + j + t) % n for t in range(sz)]  # noqa: E731
    o.ring_small = [_G(log, f"s{i}", [i]) for i in range(n)]
    o.ring_graphs = [_G(log, f"k{j}", span(j, k)) for j in range(0, n, k)]
    o.ring_mid = {sz: [_G(log, f"m{sz}", span(j, sz)) for j in range(0, n, sz)] for sz in (4, 2)}
    FusedTwoTowerStep.run(o, 19)
    assert _steps(log) == [i % n for i in range(19)] and o.ring_cursor == 19 % n
    sizes = [len(s) for _, s in log]
    assert sizes == [1, 2, 8, 8]  # 0 alone, 1-2, then 3.. as k-step graphs
