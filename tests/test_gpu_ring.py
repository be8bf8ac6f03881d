"""The production ring of the fused step (dedup one step ahead; rows looked up once updated in place
inside T1, the others by the tail launch from dX, then T3; or T2 + deferred insert, then resolver +
update + T3): bit for bit the classic step (insert in T1, every row updated
by K3), over resident batches with dropped ids, ids past N, repeated rows (2..30 lookups) and hot
rows (> 30), through HIP graphs of several steps and eagerly."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _batches(N, B, n, seed, device):
    g = torch.Generator().manual_seed(seed)
    out = []
    for s in range(n):
        cols = [torch.randint(0, 2 * x, (B,), generator=g) for x in N]
        cols[0][torch.rand(B, generator=g) < 0.03] = 0
        cols[1][:5] = 17 + s % 2         # a row repeated 5 times (K3's narrow path)
        cols[1][100:160] = 12_345        # a hot row (60 lookups: K3's hot role)
        cols[0][200:203] = cols[0][300]  # a repeated user row
        out.append(([c.to(device) for c in cols], torch.randint(0, 2, (B,), generator=g).to(torch.int32).to(device)))
    return out


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("mode", ["graph", "eager", "graph_two_launch_tail"])
def test_ring_equals_classic_step(device, D, mode):
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    N, B = [30_000, 50_000], 2048
    batches = _batches(N, B, 6, seed=D, device=device)
    a = FusedTwoTowerStep(N, [D, D], [0], [1], [128, 64], B, device, seed=2)
    b = FusedTwoTowerStep(N, [D, D], [0], [1], [128, 64], B, device, seed=2)
    assert a.ring_supported()
    a.ring_tail = mode != "graph_two_launch_tail"
    a.capture_ring(batches, steps_per_graph=2)
    if mode != "eager":
        a.run(3)
        a.run(3)  # continues at the cursor (mixed big / small graphs)
    else:
        a.run_eager(6)
    for cols, lab in batches:
        b.load_batch(cols, lab)
        b.step()
    torch.cuda.synchronize()
    assert torch.equal(a.tables.weights, b.tables.weights)
    assert torch.equal(a.tables.state, b.tables.state)
    assert torch.equal(a.params, b.params) and torch.equal(a.exp_avg, b.exp_avg)
    assert float(a.loss) == float(b.loss)
    assert torch.equal(a.logits, b.logits)


@pytest.mark.parametrize("B", [2136, 2400])
def test_ring_ragged_grid_equals_classic_step(device, B):
    """T1 grids that are not a multiple of 8 workgroups (67 tiles, the last one partial at B = 2136;
    75 at 2400): T1's XCD tile placement (xcd_remap, uneven blocks per XCD) and the insert's plain
    filing (B % 2048 != 0) — bit for bit the classic step."""
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    N = [30_000, 50_000]
    batches = _batches(N, B, 4, seed=B, device=device)
    a = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, device, seed=3)
    b = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, device, seed=3)
    assert a.ring_supported()
    a.capture_ring(batches, steps_per_graph=2)
    a.run(4)
    for cols, lab in batches:
        b.load_batch(cols, lab)
        b.step()
    torch.cuda.synchronize()
    assert torch.equal(a.tables.weights, b.tables.weights) and torch.equal(a.tables.state, b.tables.state)
    assert torch.equal(a.params, b.params) and float(a.loss) == float(b.loss)
    assert torch.equal(a.logits, b.logits)


def test_ring_large_batch_equals_classic_step(device):
    """B = 32,768 (65,536 lookups, 4096 T1 segments: past the tail list role's 2048) — the tail's slot
    role walks every claiming lookup instead of T1's list; bit for bit the classic step."""
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    N, B = [3_000_000, 5_000_000], 32768
    batches = _batches(N, B, 4, seed=32, device=device)
    a = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, device, seed=8)
    b = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, device, seed=8)
    assert a.ring_supported()
    a.capture_ring(batches, steps_per_graph=2)
    a.run(4)
    for cols, lab in batches:
        b.load_batch(cols, lab)
        b.step()
    torch.cuda.synchronize()
    assert torch.equal(a.tables.weights, b.tables.weights) and torch.equal(a.tables.state, b.tables.state)
    assert torch.equal(a.params, b.params) and float(a.loss) == float(b.loss)
    assert torch.equal(a.logits, b.logits)


def test_ring_mixed_graph_sizes(device):
    """capture_ring(k = 4) also captures aligned 2-step graphs; run(3) + run(2) replays a 2-step
    graph, single steps and a 4-step one; align_ring() regroups the graphs from the cursor; the
    8 steps train bit for bit like 8 classic steps."""
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    N, B = [30_000, 50_000], 2048
    batches = _batches(N, B, 8, seed=5, device=device)
    a = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, device, seed=2)
    b = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, device, seed=2)
    a.capture_ring(batches, steps_per_graph=4)
    assert sorted(a.ring_mid) == [2]
    a.run(3)
    a.run(2)
    a.align_ring(3)  # grouping for 3 steps from the cursor (5) is the current one: 1 step, then 2
    assert a.ring_offset == 0
    a.run(3)
    for cols, lab in batches:
        b.load_batch(cols, lab)
        b.step()
    torch.cuda.synchronize()
    assert a.ring_cursor == 0
    assert torch.equal(a.tables.weights, b.tables.weights) and torch.equal(a.tables.state, b.tables.state)
    assert torch.equal(a.params, b.params) and float(a.loss) == float(b.loss)


def test_ring_extreme_skew(device):
    """Every item lookup of a batch on ONE row (8192 lookups: a hot row split over a team of
    workgroups, its insert merged in LDS per workgroup), a few hundred distinct rows in another
    batch (rows of 2..30 and > 30 lookups), user ids uniform: the ring equals the classic step bit
    for bit over 4 steps in graphs."""
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    N, B = [3_000_000, 5_000_000], 8192
    g = torch.Generator().manual_seed(11)
    batches = []
    for s in range(4):
        cols = [torch.randint(1, N[0], (B,), generator=g), torch.randint(1, N[1], (B,), generator=g)]
        if s % 2 == 0:
            cols[1][:] = 4_242_424 + s             # one row, B lookups
        else:
            cols[1] = torch.randint(1, 300, (B,), generator=g)  # ~300 rows, ~27 lookups each
        lab = torch.randint(0, 2, (B,), generator=g).to(torch.int32)
        batches.append(([c.to(device) for c in cols], lab.to(device)))
    a = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, device, seed=3)
    b = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, device, seed=3)
    a.capture_ring(batches, steps_per_graph=2)
    a.run(4)
    for cols, lab in batches:
        b.load_batch(cols, lab)
        b.step()
    torch.cuda.synchronize()
    assert torch.equal(a.tables.weights, b.tables.weights) and torch.equal(a.tables.state, b.tables.state)
    assert torch.equal(a.params, b.params) and float(a.loss) == float(b.loss)


def test_ring_one_row_batch_vs_formula(device):
    """A batch whose 8192 item lookups all hit ONE row: the row's row-wise Adagrad step (gradient =
    the sum of the 8192 dX rows T1 left in gpooled, summed by a team of workgroups) against the
    formula in float64 on the host (rtol 1e-4: the team's summation order is not the host's)."""
    import numpy as np

    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    N, B, D, lr, row = [3_000_000, 5_000_000], 8192, 128, 0.01, 4_242_424
    g = torch.Generator().manual_seed(12)
    batches = []
    for s in range(2):
        cols = [torch.randint(1, N[0], (B,), generator=g), torch.full((B,), row + s, dtype=torch.int64)]
        batches.append(([c.to(device) for c in cols], torch.randint(0, 2, (B,), generator=g).to(torch.int32).to(device)))
    st = FusedTwoTowerStep(N, [D, D], [0], [1], [128, 64], B, device, seed=4, lr_emb=lr)
    w0 = st.tables.table_view(1)[row].double().cpu().clone()
    s0 = float(st.tables.state_view(1)[row])
    st.capture_ring(batches, steps_per_graph=2)
    st.run(1)
    torch.cuda.synchronize()
    G = st.gpooled[:, D:2 * D].double().cpu().sum(0)
    s1 = s0 + float((G * G).mean())
    w1 = w0 - lr * G / (np.sqrt(s1) + 1e-10)
    np.testing.assert_allclose(float(st.tables.state_view(1)[row]), s1, rtol=1e-4)
    np.testing.assert_allclose(st.tables.table_view(1)[row].double().cpu().numpy(), w1.numpy(), rtol=1e-4, atol=1e-7)
