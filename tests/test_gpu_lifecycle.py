"""SURVEY.md 8(f) rows 2-4 on the GPU: the reference-format checkpoint of the fused steps (save ->
load -> identical training; loads into the torchrec-shim TwoTower the way get_mlflow_model does,
03_model_training.py:1015-1054), the forward-only evaluation (03:504-566: AUROC vs scikit-learn,
the reference's loss averaging) and the embedding export (03:1056-1122: every table row through its
tower, ids labelled i + 1) against the oracle."""
import numpy as np
import pytest
import torch
from sklearn.metrics import roc_auc_score

from oracle import ref

pytestmark = pytest.mark.gpu

N = [3000, 5000]
D, B, LAYERS = 64, 512, [128, 64]


def _batches(n, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        cols = [torch.randint(0, 2 * x, (B,), generator=g) for x in N]
        out.append((cols, torch.randint(0, 2, (B,), generator=g).to(torch.int32)))
    return out


def _step(device, seed, precision="bf16"):
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    return FusedTwoTowerStep(N, [D, D], [0], [1], LAYERS, B, device, seed=seed, precision=precision)


def _train(st, batches, device):
    for cols, lab in batches:
        st.load_batch([c.to(device) for c in cols], lab.to(device))
        st.step()


def test_checkpoint_round_trip_resumes_bit_exact(device):
    from two_tower_recommender_model_amd import lifecycle as lc

    a = _step(device, 1)
    _train(a, _batches(2, 0), device)
    sd = lc.fused_state_dict(a)
    opt = lc.fused_optimizer_state(a)
    assert "two_tower.ebc.embedding_bags.t_user_id.weight" in sd
    assert "two_tower.candidate_proj._mlp.1._linear.bias" in sd
    assert sd["two_tower.ebc.embedding_bags.t_product_id.weight"].shape == (N[1], D)
    b = _step(device, 99)  # other initial weights
    lc.load_fused_state_dict(b, {k: v.cpu() for k, v in sd.items()})
    lc.load_fused_optimizer_state(b, opt)
    more = _batches(3, 7)
    _train(a, more, device)
    _train(b, more, device)
    torch.cuda.synchronize()
    assert torch.equal(a.tables.weights, b.tables.weights)
    assert torch.equal(a.tables.state, b.tables.state)
    assert torch.equal(a.params, b.params)
    assert float(a.loss) == float(b.loss)


def test_checkpoint_loads_into_reference_two_tower(device):
    """get_mlflow_model: strip "two_tower." (k[10:]), EBC + TwoTower on the torchrec API, load."""
    from two_tower_recommender_model_amd import lifecycle as lc
    from two_tower_recommender_model_amd.task import TwoTower
    from two_tower_recommender_model_amd.torchrec.modules.embedding_configs import EmbeddingBagConfig
    from two_tower_recommender_model_amd.torchrec.modules.embedding_modules import EmbeddingBagCollection
    from two_tower_recommender_model_amd.torchrec.sparse.jagged_tensor import KeyedJaggedTensor

    st = _step(device, 3, precision="fp32")
    _train(st, _batches(2, 1), device)
    sd = {k[10:]: v for k, v in lc.fused_state_dict(st).items()}
    cfgs = [EmbeddingBagConfig(name=f"t_{f}", embedding_dim=D, num_embeddings=n, feature_names=[f])
            for f, n in zip(("user_id", "product_id"), N)]
    tt = TwoTower(EmbeddingBagCollection(tables=cfgs, device=device), LAYERS, device=device)
    tt.load_state_dict(sd)
    cols, lab = _batches(1, 5)[0]
    v, l, o = ref.kjt_build([c.numpy() for c in cols], N)
    kjt = KeyedJaggedTensor(["user_id", "product_id"], torch.from_numpy(v).to(device),
                            lengths=torch.from_numpy(l).to(device), stride=B)
    with torch.no_grad():
        q, c = tt(kjt)
    logits_ref = (q * c).sum(1)
    _, logits = st.eval_step([x.to(device) for x in cols], lab.to(device))
    np.testing.assert_allclose(logits.cpu().numpy(), logits_ref.float().cpu().numpy(), rtol=2e-2, atol=2e-3)


def test_evaluate_auroc_and_reference_loss_average(device):
    from two_tower_recommender_model_amd import lifecycle as lc

    st = _step(device, 4, precision="fp32")
    _train(st, _batches(3, 2), device)
    w0 = st.tables.weights.clone()
    p0 = st.params.clone()
    ev = _batches(4, 11)
    res = lc.evaluate_fused(st, [([c.to(device) for c in cols], lab.to(device)) for cols, lab in ev])
    # forward only: nothing trained
    assert torch.equal(st.tables.weights, w0) and torch.equal(st.params, p0)
    # oracle forward (fp32) of the same state on every batch
    s0 = ref.TwoTowerState(
        tables=[st.tables.table_view(t).cpu() for t in range(2)], states=[torch.zeros(n) for n in N],
        feature_table=[0, 1], query_features=[0], cand_features=[1], dims=[D, D],
        query_layers=[(w.cpu(), b.cpu()) for w, b in zip(st.qW, st.qb)],
        cand_layers=[(w.cpu(), b.cpu()) for w, b in zip(st.cW, st.cb)])
    losses, logits_all, labels_all = [], [], []
    for cols, lab in ev:
        v, _, o = ref.kjt_build([c.numpy() for c in cols], N)
        pooled = ref.pooled_fwd(s0.tables, [0, 1], torch.from_numpy(v).to(torch.int64), torch.from_numpy(o), B)
        q = ref.mlp_fwd(pooled[:, :D], s0.query_layers)
        c = ref.mlp_fwd(pooled[:, D:], s0.cand_layers)
        logit, loss = ref.dot_bce(q, c, lab)
        losses.append(float(loss))
        logits_all.append(logit.numpy())
        labels_all.append(lab.numpy())
    # the reference divides the SUM of batch-mean losses by the number of samples (03:550-559)
    assert res["avg_loss"] == pytest.approx(sum(losses) / (len(ev) * B), rel=1e-4)
    assert res["mean_loss"] == pytest.approx(np.mean(losses), rel=1e-4)
    want_auc = roc_auc_score(np.concatenate(labels_all), 1 / (1 + np.exp(-np.concatenate(logits_all))))
    assert res["auroc"] == pytest.approx(want_auc, abs=2e-3)
    assert res["batches"] == 4 and res["samples"] == 4 * B


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-5), ("bf16", 2e-2)])
def test_export_embeddings_vs_oracle(device, precision, tol):
    from two_tower_recommender_model_amd import lifecycle as lc

    st = _step(device, 5)
    _train(st, _batches(1, 3), device)
    for tower, t, layers in (("candidate", 1, list(zip(st.cW, st.cb))), ("query", 0, list(zip(st.qW, st.qb)))):
        ids, emb = lc.export_fused(st, tower=tower, chunk=1000, precision=precision)
        assert torch.equal(ids.cpu(), torch.arange(1, N[t] + 1))  # the reference's labels (03:1168)
        want = ref.mlp_fwd(st.tables.table_view(t).cpu(), [(w.cpu(), b.cpu()) for w, b in layers])
        got = emb.cpu()
        assert got.shape == (N[t], LAYERS[-1])
        err = (got - want).abs().max() / want.abs().max()
        assert float(err) < tol, float(err)


def test_export_matches_reference_process_embeddings_on_shim(device):
    """create_keyed_jagged_tensor + process_embeddings (03:1056-1117) restated on the torchrec shim:
    a KJT with one bag per table row of the looked-up key equals the fused export."""
    from two_tower_recommender_model_amd import lifecycle as lc
    from two_tower_recommender_model_amd.task import TwoTower
    from two_tower_recommender_model_amd.torchrec.modules.embedding_configs import EmbeddingBagConfig
    from two_tower_recommender_model_amd.torchrec.modules.embedding_modules import EmbeddingBagCollection
    from two_tower_recommender_model_amd.torchrec.sparse.jagged_tensor import KeyedJaggedTensor

    st = _step(device, 6, precision="fp32")
    sd = {k[10:]: v for k, v in lc.fused_state_dict(st).items()}
    M = 2000
    cfgs = [EmbeddingBagConfig(name=f"t_{f}", embedding_dim=D, num_embeddings=M, feature_names=[f])
            for f in ("user_id", "product_id")]
    tt = TwoTower(EmbeddingBagCollection(tables=cfgs, device=device), LAYERS, device=device)
    sd = {k: (v[:M] if "embedding_bags" in k else v) for k, v in sd.items()}
    tt.load_state_dict(sd)
    values = torch.arange(M, device=device)
    lengths = torch.tensor([0] * M + [1] * M, device=device, dtype=torch.int32)  # key 'product_id'
    kjt = KeyedJaggedTensor(keys=["user_id", "product_id"], values=values, lengths=lengths)
    with torch.no_grad():
        want = tt.candidate_proj(tt.ebc(kjt)["product_id"])
    _, got = lc.export_embeddings(sd["ebc.embedding_bags.t_product_id.weight"],
                                  [(tt.candidate_proj._mlp[i]._linear.weight.detach(),
                                    tt.candidate_proj._mlp[i]._linear.bias.detach()) for i in range(2)],
                                  precision="bf16")
    np.testing.assert_allclose(got.cpu().numpy(), want.float().cpu().numpy(), rtol=3e-2, atol=3e-3)


def test_sharded_gathered_checkpoint(device):
    """Sharded step (2 ranks as threads): the gathered state dict on rank 0 is the union of the
    shards and loads into a 3-rank layout (each rank keeps its rows)."""
    import threading

    from two_tower_recommender_model_amd.sharded import FusedShardedTwoTowerStep, ThreadComm

    def run(W, fn):
        errs = []

        def wrap(r):
            try:
                fn(r)
            except BaseException as e:  # noqa: BLE001
                errs.append(e)

        th = [threading.Thread(target=wrap, args=(r,)) for r in range(W)]
        [t.start() for t in th]
        [t.join(timeout=120) for t in th]
        if errs:
            raise errs[0]

    comms = ThreadComm.group(2)
    steps = [None, None]
    out = {}

    def build(r):
        steps[r] = FusedShardedTwoTowerStep(comms[r], N, D, LAYERS, B, device, seed=2,
                                            sharding=("row_wise", "table_wise"), tw_owners=[0, 1])

    def gather(r):
        out[r] = steps[r].gathered_state_dict()

    run(2, build)
    run(2, gather)
    sd = out[0]
    assert out[1] == {}
    for f, name in enumerate(("user_id", "product_id")):
        full = sd[f"two_tower.ebc.embedding_bags.t_{name}.weight"].cpu()
        for r in range(2):
            lo, n = steps[r].spans(f)[r]
            assert torch.equal(full[lo:lo + n], steps[r].tables.table_view(f)[:n].cpu())
    comms3 = ThreadComm.group(3)
    steps3 = [None] * 3

    def build3(r):
        steps3[r] = FusedShardedTwoTowerStep(comms3[r], N, D, LAYERS, B, device, seed=9)
        steps3[r].load_state_dict(sd)

    run(3, build3)
    for r in range(3):
        for f, name in enumerate(("user_id", "product_id")):
            lo, n = steps3[r].spans(f)[r]
            assert torch.equal(steps3[r].tables.table_view(f)[:n].cpu(),
                               sd[f"two_tower.ebc.embedding_bags.t_{name}.weight"][lo:lo + n].cpu())
        assert torch.equal(steps3[r].params, steps[0].params)
