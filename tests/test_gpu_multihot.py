"""The fused step on multi-hot KJT input (FusedTwoTowerStep(max_lookups=...), SURVEY 8(d) config 5
shape at test size) against the oracle's train_step (torch CPU fp32 embedding_bag sum, towers, BCE,
row-wise Adagrad on touched rows, Adam): bags of 0..9 ids (empty bags included), ids in range as a
KJT carries them (03_model_training.py:367-371, :417).

Tolerances: pooled embeddings (fp32 sums; torch CPU embedding_bag adds in its own order) rtol 1e-5, atol 1e-6 x max bag length; fp32 parity mode loss/logits
rtol 1e-4 and updated tables atol 1e-5 over 3 steps; bf16 towers: pooled exact-order sums as above,
loss rtol 2e-2 on the first step."""
import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


def _kjt(rng, B, N, maxlen, hot=False):
    lengths = rng.integers(0, maxlen + 1, 2 * B).astype(np.int32)
    vals = []
    for i in range(2 * B):
        n = N[i // B]
        v = (rng.zipf(1.5, lengths[i]) - 1) % n if hot else rng.integers(0, n, lengths[i])
        vals.extend(v.tolist())
    return np.asarray(vals, np.int64), ref.complete_cumsum(lengths)


def _state(st, N, D):
    return ref.TwoTowerState(
        tables=[st.tables.table_view(0).cpu().clone(), st.tables.table_view(1).cpu().clone()],
        states=[torch.zeros(n) for n in N], feature_table=[0, 1], query_features=[0], cand_features=[1],
        dims=[D, D], query_layers=[(w.cpu().clone(), b.cpu().clone()) for w, b in zip(st.qW, st.qb)],
        cand_layers=[(w.cpu().clone(), b.cpu().clone()) for w, b in zip(st.cW, st.cb)])


@pytest.mark.parametrize("hot", [False, True], ids=["uniform", "zipf"])
def test_multihot_step_fp32_vs_oracle(device, hot):
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    rng = np.random.default_rng(21 if hot else 20)
    B, D, layers, N = 128, 64, [64, 32], [300, 500]
    batches = [_kjt(rng, B, N, 9, hot) for _ in range(3)]
    cap = max(v.size for v, _ in batches)
    st = FusedTwoTowerStep(N, [D, D], [0], [1], layers, B, device, lr_emb=0.02, lr_dense=0.01, precision="fp32",
                           seed=4, max_lookups=cap)
    s0 = _state(st, N, D)
    g = torch.Generator().manual_seed(9)
    for v, o in batches:
        labels = torch.randint(0, 2, (B,), generator=g).to(torch.int32)
        st.load_kjt(torch.from_numpy(v).to(device), torch.from_numpy(o).to(device), labels.to(device))
        st.step()
        torch.cuda.synchronize()
        loss, logits, pooled, _ = ref.train_step(s0, torch.from_numpy(v), torch.from_numpy(o), B, labels, 0.02, 0.01)
        np.testing.assert_allclose(st.pooled.cpu().numpy(), pooled.numpy(), rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(st.logits.cpu().numpy(), logits.numpy(), rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(float(st.loss), float(loss), rtol=1e-4)
    for t in range(2):
        np.testing.assert_allclose(st.tables.table_view(t).cpu().numpy(), s0.tables[t].numpy(), rtol=0, atol=1e-5)
        np.testing.assert_allclose(st.tables.state_view(t).cpu().numpy(), s0.states[t].numpy(), rtol=1e-4, atol=1e-9)


def test_multihot_step_bf16_graph(device):
    """bf16 fused towers, one HIP graph per resident batch (capture_pool_kjt), first step vs the
    oracle; a replay of the same graph sequence from the same state is bitwise reproducible."""
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    rng = np.random.default_rng(22)
    B, D, layers, N = 256, 128, [128, 64], [2000, 3000]
    host = [_kjt(rng, B, N, 9) for _ in range(2)]
    g = torch.Generator().manual_seed(2)
    labels = [torch.randint(0, 2, (B,), generator=g).to(torch.int32) for _ in host]
    batches = [(torch.from_numpy(v).to(device), torch.from_numpy(o).to(device), lab.to(device))
               for (v, o), lab in zip(host, labels)]
    cap = max(v.size for v, _ in host)

    def run():
        st = FusedTwoTowerStep(N, [D, D], [0], [1], layers, B, device, lr_emb=0.02, lr_dense=0.01, seed=5,
                               max_lookups=cap, materialize_pooled=True)
        assert st.towers is not None and st.gather_kjt  # the fused bf16 tower kernels, sum pool inside T1
        s0 = _state(st, N, D)
        st.capture_pool_kjt(batches)
        st.pool_graphs[0].replay()
        torch.cuda.synchronize()
        first = (st.pooled.cpu().clone(), float(st.loss))
        st.pool_graphs[1].replay()
        torch.cuda.synchronize()
        return st, s0, first

    st, s0, (pooled, loss) = run()
    v, o = host[0]
    want_loss, _, want_pooled, _ = ref.train_step(s0, torch.from_numpy(v), torch.from_numpy(o), B, labels[0], 0.02,
                                                  0.01)
    np.testing.assert_allclose(pooled.numpy(), want_pooled.numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(loss, float(want_loss), rtol=2e-2)
    st2, _, _ = run()
    assert torch.equal(st.tables.weights, st2.tables.weights) and torch.equal(st.params, st2.params)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_config3_shape_step_vs_oracle(device, precision):
    """SURVEY 8(d) config 3 shape at test size: 8 single-hot features per tower (16 tables), towers
    over the concatenation (in_size = 8 x D = 512), ids through the reference transform (id 0
    dropped, id mod N). fp32 parity mode: 2 steps vs the oracle (pooled rows exact on the first step,
    then atol 1e-5; loss rtol 1e-4, tables atol 1e-5); bf16 fused towers: the first step's pooled rows
    exactly and its loss rtol 2e-2."""
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    F, B, D, layers = 16, 64, 64, [64, 32]
    N = [200 + 37 * f for f in range(F)]
    st = FusedTwoTowerStep(N, [D] * F, list(range(8)), list(range(8, 16)), layers, B, device, lr_emb=0.02,
                           lr_dense=0.01, precision=precision, seed=7, materialize_pooled=True)
    if precision == "bf16":
        assert st.towers is not None
    s0 = ref.TwoTowerState(
        tables=[st.tables.table_view(f).cpu().clone() for f in range(F)], states=[torch.zeros(n) for n in N],
        feature_table=list(range(F)), query_features=list(range(8)), cand_features=list(range(8, 16)),
        dims=[D] * F, query_layers=[(w.cpu().clone(), b.cpu().clone()) for w, b in zip(st.qW, st.qb)],
        cand_layers=[(w.cpu().clone(), b.cpu().clone()) for w, b in zip(st.cW, st.cb)])
    g = torch.Generator().manual_seed(3)
    for step in range(2 if precision == "fp32" else 1):
        cols = [torch.randint(0, 2 * n, (B,), generator=g) for n in N]
        for c in cols:
            c[:3] = 0  # dropped ids: empty bags
        labels = torch.randint(0, 2, (B,), generator=g).to(torch.int32)
        st.load_batch([c.to(device) for c in cols], labels.to(device))
        st.step()
        torch.cuda.synchronize()
        v, _, o = ref.kjt_build([c.numpy() for c in cols], N)
        loss, logits, pooled, _ = ref.train_step(s0, torch.from_numpy(v), torch.from_numpy(o), B, labels, 0.02, 0.01)
        if step == 0:  # a gather of identical tables: exact; later steps gather updated rows (atol 1e-5)
            np.testing.assert_array_equal(st.pooled.cpu().numpy(), pooled.numpy())
        else:
            np.testing.assert_allclose(st.pooled.cpu().numpy(), pooled.numpy(), rtol=0, atol=1e-5)
        np.testing.assert_allclose(float(st.loss), float(loss), rtol=1e-4 if precision == "fp32" else 2e-2)
    if precision == "fp32":
        for f in range(F):
            np.testing.assert_allclose(st.tables.table_view(f).cpu().numpy(), s0.tables[f].numpy(), rtol=0, atol=1e-5)


@pytest.mark.parametrize("k", [1, 2, 4], ids=["graph1", "graph2", "graph4-aligned"])
@pytest.mark.parametrize("hot", [False, True], ids=["uniform", "zipf"])
def test_multihot_pipelined_grouping_bitwise(device, hot, k):
    """The pipelined pool (capture_pool_kjt(ahead=True): batch i+1's backward grouping built on the
    side stream during step i, two alternating workspaces) trains exactly like the unpipelined
    pool: 4 batches x 2 cycles of graph replays, tables / row-wise state / tower parameters / loss
    bitwise equal; then 3 eager pipelined steps (pool_step_eager) continue bitwise like 3 more
    unpipelined graph replays. Zipf ids exercise the hot-row kernels; k = 2 replays graphs of two
    pipelined steps where the cursor allows (replay_pool); k = 4 regroups the graphs for a run of 6
    steps after 1 (align_pool: graphs grouped from pool position 3, the run's 2 remainder steps
    first as a 2-step graph, then one 4-step graph), around single-step graphs."""
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    rng = np.random.default_rng(23 if hot else 24)
    B, D, layers, N = 256, 128, [128, 64], [2000, 3000]
    host = [_kjt(rng, B, N, 9, hot) for _ in range(4)]
    g = torch.Generator().manual_seed(5)
    batches = [(torch.from_numpy(v).to(device), torch.from_numpy(o).to(device),
                torch.randint(0, 2, (B,), generator=g).to(torch.int32).to(device)) for v, o in host]
    cap = max(v.size for v, _ in host)

    def make():
        return FusedTwoTowerStep(N, [D, D], [0], [1], layers, B, device, lr_emb=0.02, lr_dense=0.01, seed=6,
                                 max_lookups=cap)

    ref_st, pipe = make(), make()
    ref_st.capture_pool_kjt(batches)
    pipe.capture_pool_kjt(batches, ahead=True, steps_per_graph=k)  # k > 1: graphs of k steps too
    for i in range(8):
        ref_st.pool_graphs[i % 4].replay()
    if k == 4:
        pipe.align_pool(6, after=1)
        assert pipe.pool_offset == 3 and set(pipe.pool_mid) == {2}
        pipe.replay_pool(1)  # position 0 alone
        pipe.replay_pool(6)  # 1-2 as a 2-step graph, 3, 0, 1, 2 as a 4-step graph
        pipe.replay_pool(1)
    else:
        pipe.replay_pool(8)
    torch.cuda.synchronize()
    for a, b in ((ref_st.tables.weights, pipe.tables.weights), (ref_st.tables.state, pipe.tables.state),
                 (ref_st.params, pipe.params), (ref_st.loss, pipe.loss)):
        assert torch.equal(a, b)
    for i in range(3):
        ref_st.pool_graphs[i].replay()
        pipe.pool_step_eager()
    torch.cuda.synchronize()
    assert torch.equal(ref_st.tables.weights, pipe.tables.weights) and torch.equal(ref_st.params, pipe.params)
    assert torch.equal(ref_st.tables.state, pipe.tables.state)


@pytest.mark.parametrize("D,id_dtype,empty", [(64, torch.int64, False), (128, torch.int64, False),
                                               (128, torch.int32, False), (128, torch.int64, True)],
                         ids=["d64", "d128", "d128-int32", "d128-empty-batch"])
def test_multihot_pool_inside_t1_bitwise(device, D, id_dtype, empty):
    """tt_tower_fwd_bwd_kjt (the sum pool of every bag inside T1) against tt_pooled_fwd followed by
    the unfused T1 on the same KJT: pooled rows, logits, dX, loss, and after 3 eager steps the
    tables, row-wise state and tower parameters, all bitwise (the rows are added in bag order from
    zero in both). Bags of 0..40 ids (empty bags, bags longer than one 32-id chunk), B not a multiple
    of the 32-row tile."""
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    rng = np.random.default_rng(31 + D)
    B, N = 200, [3000, 5000]
    batches = [_kjt(rng, B, N, 40) for _ in range(3)]
    if empty:  # a batch whose every bag is empty (all ids dropped upstream): zero rows, no lookups
        batches[1] = (np.zeros(0, np.int64), np.zeros(2 * B + 1, np.int32))
    cap = max(1, max(v.size for v, _ in batches))
    g = torch.Generator().manual_seed(4)
    labels = [torch.randint(0, 2, (B,), generator=g).to(torch.int32).to(device) for _ in batches]
    outs = []
    for fuse in (False, True):
        st = FusedTwoTowerStep(N, [D, D], [0], [1], [128, 64], B, device, lr_emb=0.02, lr_dense=0.01, seed=6,
                               max_lookups=cap, fuse_gather=fuse, materialize_pooled=True, id_dtype=id_dtype)
        assert st.gather_kjt == fuse and st.towers is not None
        per = []
        for (v, o), lab in zip(batches, labels):
            st.load_kjt(torch.from_numpy(v).to(id_dtype).to(device), torch.from_numpy(o).to(device), lab)
            st.step()
            torch.cuda.synchronize()
            per.append([x.cpu().clone() for x in (st.pooled, st.logits, st.gpooled, st.loss)])
        outs.append((per, st.tables.weights.cpu(), st.tables.state.cpu(), st.params.cpu()))
    (p0, w0, s0, q0), (p1, w1, s1, q1) = outs
    for a_, b_ in zip(p0, p1):
        for x, y in zip(a_, b_):
            assert torch.equal(x, y)
    assert torch.equal(w0, w1) and torch.equal(s0, s1) and torch.equal(q0, q1)
