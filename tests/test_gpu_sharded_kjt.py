"""The capturable multi-hot sharded step (two_tower_recommender_model_amd/sharded_kjt.py,
csrc/shard_kjt.hip; BASELINE config 5's shape: users table-wise, items row-wise, bags of several ids):

* the route / unpack / partial-sum / gradient-pack kernels against a restatement of TorchRec's
  input_dist (block_bucketize by row block, table-wise owner) and output_dist (reduce-scatter =
  sum of the owners' partial pools), bit-exact for the integer work;
* W = 1 against the single-GPU multi-hot fused step (FusedTwoTowerStep(max_lookups=...));
* W = 2, 3, 4 ranks as threads over an in-process all-to-all (ThreadComm) against the oracle (and
  W = 2 at BASELINE config 5's table sizes and batch): each
  rank's pooled tower input against the oracle's sum pools of the tables before the step (fp32
  summation-order bound), its towers element-wise against the fp64 emulation of the bf16 kernels
  on ITS OWN batch, every touched row against the oracle's row-wise Adagrad over the union of the
  emulated bag gradients (each lookup of a bag adds the bag's gradient), and Adam on the fixed-order
  sum of the ranks' tower gradients, identical on every rank.
"""
import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


def _kjt(N, B, maxlen, gen, empty_frac=0.1):
    """Key-major multi-hot KJT over len(N) features: lengths U{1..maxlen} (some empty), ids in range."""
    lengths, vals = [], []
    for n in N:
        l = torch.randint(1, maxlen + 1, (B,), generator=gen)
        l[torch.rand(B, generator=gen) < empty_frac] = 0
        lengths.append(l)
        vals.append(torch.randint(0, n, (int(l.sum()),), generator=gen))
    lengths = torch.cat(lengths).to(torch.int32)
    offsets = torch.zeros(lengths.numel() + 1, dtype=torch.int32)
    offsets[1:] = torch.cumsum(lengths, 0)
    return torch.cat(vals).to(torch.int32), offsets, lengths


def _route_want(values, offsets, B, N, sharding, owners, W, cap):
    """input_dist restated: per destination d, lengths [F][B] of the ids d owns (row-wise: id //
    ceil(N/W); table-wise: the owner) and those ids' rows in d's shard, in (feature, bag, position)
    order (fbgemm block_bucketize_sparse_features / TorchRec TW grouping)."""
    F = len(N)
    v, o = values.numpy().astype(np.int64), offsets.numpy()
    lens = np.zeros((W, F * B), np.int32)
    ids = [[] for _ in range(W)]
    for f in range(F):
        bs = -(-N[f] // W)
        for b in range(B):
            for x in v[o[f * B + b]:o[f * B + b + 1]]:
                d = int(x // bs) if sharding[f] == "row_wise" else owners[f]
                lens[d, f * B + b] += 1
                ids[d].append(int(x - d * bs) if sharding[f] == "row_wise" else int(x))
    return lens, ids


@pytest.mark.parametrize("W,sharding,owners", [(1, ("table_wise", "row_wise"), (0, 0)),
                                               (3, ("table_wise", "row_wise"), (2, 0)),
                                               (4, ("row_wise", "row_wise"), (0, 0)),
                                               (2, ("table_wise", "table_wise"), (1, 0))])
def test_kjt_route_unpack_partials_vs_restatement(device, W, sharding, owners):
    import ctypes as C

    from two_tower_recommender_model_amd import _lib
    from two_tower_recommender_model_amd._lib import ptr

    gen = torch.Generator().manual_seed(W)
    N, B, D = [1000, 1777], 300, 32
    F = len(N)
    values, offsets, _ = _kjt(N, B, 7, gen)
    lens, ids = _route_want(values, offsets, B, N, sharding, owners, W, None)
    need = max(len(x) for x in ids)
    lib = _lib.load()
    dv, do = values.to(device), offsets.to(device)  # kept alive across the launches
    for cap in (need, max(0, need - 1)):
        stride = F * B + cap + 5
        send = torch.full((W * stride,), -7, dtype=torch.int32, device=device)
        flags = torch.zeros(2, dtype=torch.int32, device=device)
        ws = torch.empty(lib.tt_kjt_route_workspace_bytes(F, B, W), dtype=torch.uint8, device=device)
        bs = [-(-n // W) if s == "row_wise" else 0 for n, s in zip(N, sharding)]
        _lib.check(lib.tt_kjt_route(F, B, ptr(dv), _lib.TT_I32, ptr(do),
                                    (C.c_int64 * F)(*N), (C.c_int64 * F)(*bs), (C.c_int32 * F)(*owners), W, cap, stride,
                                    ptr(send), ptr(flags), ptr(ws), ws.numel(), _lib.stream_handle(device)))
        torch.cuda.synchronize()
        assert int(flags[0]) == (cap < need) and int(flags[1]) == 0
        s = send.cpu().numpy().reshape(W, stride)
        if cap < need:
            # an overflowing block keeps the ids that fit and sends lengths that agree with them; the
            # owner's unpack then stays inside its W * cap values (guard past them untouched)
            for d in range(W):
                kept = s[d, :F * B]
                assert kept.sum() == min(cap, len(ids[d])) and (kept <= lens[d]).all()
                np.testing.assert_array_equal(s[d, F * B:F * B + kept.sum()], ids[d][:kept.sum()])
                recv = torch.from_numpy(np.tile(s[d], W)).to(device)
                Fr = F
                lo = torch.empty(W * Fr * B, dtype=torch.int32, device=device)
                oo = torch.empty(W * Fr * B + 1, dtype=torch.int32, device=device)
                vo = torch.full((W * cap + 4096,), -1, dtype=torch.int32, device=device)
                uw = torch.empty(max(256, lib.tt_kjt_unpack_workspace_bytes(W, Fr, B)), dtype=torch.uint8,
                                 device=device)
                _lib.check(lib.tt_kjt_unpack(W, F, B, ptr(recv), stride, cap, (C.c_int32 * Fr)(*range(F)), Fr,
                                             ptr(lo), ptr(oo), ptr(vo), ptr(uw), uw.numel(),
                                             _lib.stream_handle(device)))
                torch.cuda.synchronize()
                assert int(oo[-1]) <= W * cap
                assert (vo[W * cap:] == -1).all()
            continue
        for d in range(W):
            np.testing.assert_array_equal(s[d, :F * B], lens[d])
            np.testing.assert_array_equal(s[d, F * B:F * B + len(ids[d])], ids[d])
        # the owner side of every rank d: unpack the blocks every source sent it (here: W copies of
        # this source's block for d, i.e. the recv buffer of rank d if every rank had this batch)
        for d in range(W):
            feats = [f for f in range(F) if sharding[f] == "row_wise" or owners[f] == d]
            if not feats:
                continue
            Fr = len(feats)
            recv = torch.from_numpy(np.tile(s[d], W)).to(device)
            lo = torch.empty(W * Fr * B, dtype=torch.int32, device=device)
            oo = torch.empty(W * Fr * B + 1, dtype=torch.int32, device=device)
            vo = torch.full((W * cap + 1,), -1, dtype=torch.int32, device=device)
            uw = torch.empty(max(256, lib.tt_kjt_unpack_workspace_bytes(W, Fr, B)), dtype=torch.uint8, device=device)
            _lib.check(lib.tt_kjt_unpack(W, F, B, ptr(recv), stride, cap, (C.c_int32 * Fr)(*feats), Fr, ptr(lo),
                                         ptr(oo), ptr(vo), ptr(uw), uw.numel(), _lib.stream_handle(device)))
            torch.cuda.synchronize()
            want_l = np.tile(np.concatenate([lens[d][f * B:(f + 1) * B] for f in feats]), W)
            np.testing.assert_array_equal(lo.cpu().numpy(), want_l)
            np.testing.assert_array_equal(oo.cpu().numpy(), np.concatenate([[0], np.cumsum(want_l)]))
            np.testing.assert_array_equal(vo.cpu().numpy()[:W * len(ids[d])], np.tile(ids[d], W))
    # partial sum / gradient pack: owner d's block rows hold feature f at column k * D
    Fmax = max(len([f for f in range(F) if sharding[f] == "row_wise" or owners[f] == d]) for d in range(W))
    col = np.full((W, F), -1, np.int32)
    for d in range(W):
        for k, f in enumerate([f for f in range(F) if sharding[f] == "row_wise" or owners[f] == d]):
            col[d, f] = k * D
    strideB = B * Fmax * D + 8
    recvB = torch.randn(W * strideB, generator=gen)
    drecvB = recvB.to(device)
    out = torch.empty(B, F * D, device=device)
    oc = (C.c_int32 * (W * F))(*col.reshape(-1).tolist())
    _lib.check(lib.tt_pooled_partials_sum(W, F, B, D, ptr(drecvB), strideB, Fmax * D, oc, ptr(out),
                                          out.stride(0), _lib.stream_handle(device)))
    want = torch.zeros(B, F * D)
    blocks = recvB[:W * strideB].view(W, strideB)
    for f in range(F):
        for d in range(W):  # ascending owners: the kernel's order
            if col[d, f] >= 0:
                want[:, f * D:(f + 1) * D] += blocks[d, :B * Fmax * D].view(B, Fmax * D)[:, col[d, f]:col[d, f] + D]
    assert torch.equal(out.cpu(), want)
    g = torch.randn(B, F * D, generator=gen)
    dg = g.to(device)
    sendC = torch.zeros(W * strideB, device=device)
    _lib.check(lib.tt_pooled_grad_pack(W, F, B, D, ptr(dg), F * D, oc, ptr(sendC), strideB, Fmax * D,
                                       _lib.stream_handle(device)))
    sc = sendC.cpu().view(W, strideB)
    for d in range(W):
        for f in range(F):
            if col[d, f] >= 0:
                assert torch.equal(sc[d, :B * Fmax * D].view(B, Fmax * D)[:, col[d, f]:col[d, f] + D],
                                   g[:, f * D:(f + 1) * D])


def test_sharded_kjt_w1_vs_fused_multihot_step(device):
    """One rank (ThreadComm): the sharded multi-hot step against FusedTwoTowerStep's multi-hot step on
    the same batches — pooling, towers and the row update run the same kernels (bit-identical up to
    Adam, whose scalars come from a different launch: 1e-6 relative)."""
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep
    from two_tower_recommender_model_amd.sharded import ThreadComm
    from two_tower_recommender_model_amd.sharded_kjt import FusedShardedKJTStep

    N, B, D = [4000, 6000], 512, 128
    gen = torch.Generator().manual_seed(11)
    batches = [_kjt(N, B, 9, gen) + (torch.randint(0, 2, (B,), generator=gen).to(torch.int32),) for _ in range(3)]
    cap = max(int(v.numel()) for v, _, _, _ in batches)
    ref_step = FusedTwoTowerStep(N, [D, D], [0], [1], [128, 64], B, device, seed=4, max_lookups=cap,
                                 id_dtype=torch.int32)
    full = [ref_step.tables.table_view(f).cpu().clone() for f in range(2)]
    sh = FusedShardedKJTStep(ThreadComm.group(1)[0], N, D, [128, 64], B, device, cap=cap, full_tables=full,
                             sharding=("table_wise", "row_wise"), tw_owners=(0, 0))
    sh.params.copy_(ref_step.params)
    sh.towers.update(sh.params, do_adam=False)
    for s, (v, o, _, lab) in enumerate(batches):
        ref_step.load_kjt(v.to(device), o.to(device), lab.to(device))
        ref_step.step()
        sh.step(v.to(device), o.to(device), lab.to(device))
        torch.cuda.synchronize()
        if s == 0:  # the same parameters in: bit-identical towers
            assert torch.equal(sh.logits, ref_step.logits)
        np.testing.assert_allclose(sh.logits.cpu().numpy(), ref_step.logits.cpu().numpy(), rtol=1e-5, atol=1e-6)
    sh.check()
    for f in range(2):
        np.testing.assert_allclose(sh.tables.table_view(f).cpu().numpy(), ref_step.tables.table_view(f).cpu().numpy(),
                                   rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(sh.tables.state_view(f).cpu().numpy(), ref_step.tables.state_view(f).cpu().numpy(),
                                   rtol=1e-4, atol=1e-12)
    np.testing.assert_allclose(sh.params.cpu().numpy(), ref_step.params.cpu().numpy(), rtol=1e-5, atol=1e-7)


def _run_ranks(fns):
    import threading

    errs = []

    def wrap(fn):
        try:
            fn()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=wrap, args=(fn,)) for fn in fns]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=180)
    if errs:
        raise errs[0]


@pytest.mark.parametrize("W,sharding,owners", [(2, ("table_wise", "row_wise"), (1, 0)),
                                               (4, ("table_wise", "row_wise"), (3, 0)),
                                               (3, ("row_wise", "row_wise"), (0, 0))])
def test_sharded_kjt_threads_vs_oracle(device, W, sharding, owners):
    _threads_vs_oracle(device, W, sharding, owners, [3000, 5000], 256, 9, 2, full_init=True)


def test_sharded_kjt_threads_baseline_sizes_vs_oracle(device):
    """BASELINE config 5 at full size as W = 2 thread ranks: 50M users table-wise on rank 1, 100M
    items row-wise, B = 16,384 bags of 1..39 ids per tower and rank (~0.65M lookups a feature a
    step), both ranks' shards on the one GPU (77 GB); tables drawn on the device, the oracle fed
    the touched rows read back before each step."""
    _threads_vs_oracle(device, 2, ("table_wise", "row_wise"), (1, 0), [50_000_000, 100_000_000], 16384, 39, 2,
                       full_init=False)


def _threads_vs_oracle(device, W, sharding, owners, N, B, maxlen, nsteps, full_init):
    from tower_emul import acc_err, check_adagrad, check_towers, check_within, emulate_bounds, split_params

    from two_tower_recommender_model_amd.sharded import ThreadComm
    from two_tower_recommender_model_amd.sharded_kjt import FusedShardedKJTStep, route_counts

    D, lr, layers, F = 128, 0.02, [128, 64], 2
    gen = torch.Generator().manual_seed(50 + W)
    full = [torch.empty(n, D).uniform_(-0.05, 0.05, generator=gen) for n in N] if full_init else None
    data = [[_kjt(N, B, maxlen, gen) + (torch.randint(0, 2, (B,), generator=gen).to(torch.int32),) for _ in range(W)]
            for _ in range(nsteps)]
    for step_batches in data:  # a hot item in every rank's batch (rows summed across ranks)
        for v, o, _, _ in step_batches:
            v[int(o[B]):int(o[B]) + 5] = 4242
    cap = max(int(route_counts(v, o, B, N, sharding, owners, W).max()) for sb in data for v, o, _, _ in sb)
    comms = ThreadComm.group(W)
    ranks = [None] * W

    def build(r):
        torch.cuda.set_device(device)
        ranks[r] = FusedShardedKJTStep(comms[r], N, D, layers, B, device, cap=cap, sharding=sharding, tw_owners=owners,
                                       lr_emb=lr, full_tables=full, seed=3)

    _run_ranks([lambda r=r: build(r) for r in range(W)])
    P = ranks[0].towers.num_params
    m_ref, v_ref = [torch.zeros(P)], [torch.zeros(P)]

    def read_rows(f, u):
        w = torch.empty(u.numel(), D)
        s_ = torch.empty(u.numel())
        for st in ranks:
            lo, n = st.row_lo[f], st.local_rows[f]
            sel = (u >= lo) & (u < lo + n)
            if bool(sel.any()):
                idx = (u[sel] - lo).to(device)
                w[sel] = st.tables.table_view(f)[idx].cpu()
                s_[sel] = st.tables.state_view(f)[idx].cpu()
        return w, s_

    for s in range(nsteps):
        params0 = ranks[0].params.cpu().clone()
        uniq = []
        for f in range(F):
            ids = torch.cat([v[int(o[f * B]):int(o[(f + 1) * B])] for v, o, _, _ in data[s]]).to(torch.int64)
            uniq.append(torch.unique(ids))
        before = [read_rows(f, uniq[f]) for f in range(F)]
        torch.cuda.synchronize()

        def run(r):
            torch.cuda.set_device(device)
            v, o, _, lab = data[s][r]
            ranks[r].step(v.to(device), o.to(device), lab.to(device))
            torch.cuda.synchronize()

        _run_ranks([lambda r=r: run(r) for r in range(W)])
        _run_ranks([lambda r=r: ranks[r].check() for r in range(W)])
        rows_all, dx_all, eb_all = [[] for _ in N], [[] for _ in N], [[] for _ in N]
        tower_sum = torch.zeros(P)
        for r in range(W):
            st = ranks[r]
            v, o, lengths, lab = data[s][r]
            o64 = o.to(torch.int64)
            # (a) the pooled tower input vs the oracle's sum pools of the tables before the step
            got = st.pooled.cpu()
            for f in range(F):
                bag = torch.repeat_interleave(torch.arange(B), lengths[f * B:(f + 1) * B].to(torch.int64))
                ids = v[int(o64[f * B]):int(o64[(f + 1) * B])].to(torch.int64)
                rows = before[f][0][torch.searchsorted(uniq[f], ids)].double()
                want = torch.zeros(B, D, dtype=torch.float64).index_add_(0, bag, rows)
                l2 = torch.zeros(B, D, dtype=torch.float64).index_add_(0, bag, rows * rows).sqrt()
                n = lengths[f * B:(f + 1) * B].clamp(min=1).double()[:, None]
                check_within(got[:, f * D:(f + 1) * D], want, acc_err(l2, want, 1) * n.sqrt(), f"rank {r} pooled {f}")
                rows_all[f].append((ids, bag))
            # (b) towers vs the emulation on this rank's own batch
            prm = split_params(params0, st.in_dims, layers)
            lg, loss, dxs, gw, amb = emulate_bounds(got[:, :D], got[:, D:], prm, layers, lab)
            gpo = st.gpooled.cpu()
            sent = st.tower_grad_sent().cpu()
            glist, oo = [], 0
            for p_ in prm:
                glist.append(sent[oo:oo + p_.numel()].reshape(p_.shape) * W)
                oo += p_.numel()
            check_towers((lg, loss, dxs, gw, amb), st.logits.cpu(), [gpo[:, :D], gpo[:, D:]], glist, f"rank {r}")
            for f in range(F):
                ids, bag = rows_all[f][-1]
                dx_all[f].append(dxs[f][0][bag])
                eb_all[f].append(dxs[f][1][bag])
            tower_sum += sent
        # (c) every touched row vs the oracle's Adagrad over the union of the emulated bag gradients
        for f in range(F):
            inv = torch.searchsorted(uniq[f], torch.cat([ids for ids, _ in rows_all[f]]))
            w_got, s_got = read_rows(f, uniq[f])
            check_adagrad(w_got, s_got, before[f][0], before[f][1], inv, torch.cat(dx_all[f]), torch.cat(eb_all[f]),
                          lr, 1e-10, f"feature {f}")
        # (d) Adam on the fixed-order sum of the tower gradients; identical replicas
        p_ref = [params0.clone()]
        ref.adam(p_ref, [tower_sum], m_ref, v_ref, s + 1, 0.01)
        np.testing.assert_allclose(ranks[0].params.cpu().numpy(), p_ref[0].numpy(), rtol=1e-5, atol=1e-7)
        for r in range(1, W):
            assert torch.equal(ranks[r].params, ranks[0].params)


def test_sharded_kjt_rccl_world1_graph_equals_eager(device):
    """The three all-to-alls on RCCL, captured into HIP graphs, against eager steps (child process:
    tests/rccl_kjt_graph_check.py)."""
    from child_util import run_child

    run_child(["tests/rccl_kjt_graph_check.py"], "RCCL-KJT-GRAPH-OK", timeout=300)


def test_sharded_kjt_peer_world1_graph_equals_rccl_eager(device):
    """The three exchanges on the device-initiated PeerComm, captured, against the eager RCCL steps, bit
    for bit (the same child with TT_KJT_COMM=peer)."""
    import os

    from child_util import run_child

    run_child(["tests/rccl_kjt_graph_check.py"], "RCCL-KJT-GRAPH-OK", timeout=300,
              env=dict(os.environ, TT_KJT_COMM="peer"))
