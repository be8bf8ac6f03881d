"""The reference's own loop (DistributedModelParallel + TrainPipelineSparseDist.progress +
KeyedOptimizerWrapper(Adam) + RowWiseAdagrad in backward, 03_model_training.py:612-625, :770-829)
dispatched to the fused production ring (two_tower_recommender_model_amd/dropin.py):

* dispatch happens for the reference's two-tower shape (bf16 towers [128, 64], D 64 / 128) and the
  result is BIT-IDENTICAL to FusedTwoTowerStep's ring on the same batches (tables, Adagrad state,
  tower parameters, Adam moments, per-step logits and loss);
* against the reference's own golden trajectory (tests/golden/train_d128.npz) with the bf16
  tolerances of test_gpu_step.py;
* a smaller last batch runs the generic per-op path between fused steps on the shared storage
  (Adam step count carried both ways), a second chunk after StopIteration re-primes the ring, and
  eval mode is forward-only — against the same sequence with the dispatch off (TT_DROPIN_FUSED=0),
  bf16 tolerances;
* a bag of several ids in a later batch is reported (TTError at the chunk's end).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

FEATS = ["user_id", "product_id"]


def _reference_wiring(device, N, D, lr_emb, lr_dense, layers=(128, 64), init=None):
    """main()'s setup (03:770-829) on the torchrec shim, world size 1, no process group."""
    import two_tower_recommender_model_amd as tt

    tt.install_torchrec_alias()
    from torch.distributed.optim import _apply_optimizer_in_backward
    from torchrec.distributed import TrainPipelineSparseDist
    from torchrec.distributed.model_parallel import DistributedModelParallel
    from torchrec.modules.embedding_configs import EmbeddingBagConfig
    from torchrec.modules.embedding_modules import EmbeddingBagCollection
    from torchrec.optim.keyed import KeyedOptimizerWrapper
    from torchrec.optim.rowwise_adagrad import RowWiseAdagrad

    from two_tower_recommender_model_amd.task import TwoTower, TwoTowerTrainTask

    cfgs = [EmbeddingBagConfig(name=f"t_{f}", embedding_dim=D, num_embeddings=N[i], feature_names=[f])
            for i, f in enumerate(FEATS)]
    ebc = EmbeddingBagCollection(tables=cfgs, device=torch.device("meta"))
    two_tower = TwoTower(embedding_bag_collection=ebc, layer_sizes=list(layers), device=device)
    task = TwoTowerTrainTask(two_tower)
    _apply_optimizer_in_backward(RowWiseAdagrad, task.two_tower.ebc.parameters(), {"lr": lr_emb})
    model = DistributedModelParallel(module=task, device=device)
    if init is not None:
        sd = model.module.two_tower.state_dict()
        with torch.no_grad():
            for k, v in init.items():
                sd[k].copy_(v)
    optimizer = KeyedOptimizerWrapper(dict(model.named_parameters()), lambda ps: torch.optim.Adam(ps, lr=lr_dense))
    return model, optimizer, TrainPipelineSparseDist(model, optimizer, device)


def _kjt_batch(cols, labels, N, dtype):
    """transform_to_torchrec_batch (03:353-380), vectorised: id 0 dropped, id % N kept."""
    from torchrec.datasets.utils import Batch
    from torchrec.sparse.jagged_tensor import KeyedJaggedTensor

    vals, lens = [], []
    for c, n in zip(cols, N):
        c = c.to(torch.int64)
        keep = c != 0
        vals.append(torch.remainder(c[keep], n))
        lens.append(keep.to(torch.int32))
    v = torch.cat(vals).to(dtype)
    kjt = KeyedJaggedTensor.from_lengths_sync(FEATS, v, torch.cat(lens))
    return Batch(dense_features=torch.zeros(1), sparse_features=kjt, labels=labels.to(torch.int32))


def _synthetic(N, B, n, seed, dtype=torch.int64):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        cols = []
        for Ni in N:
            c = torch.randint(0, 2 * Ni, (B,), generator=g)  # ids past N wrap (id % N), some exactly N
            c[torch.rand(B, generator=g) < 0.05] = 0          # dropped
            c[:3] = Ni                                        # id N -> row 0, kept
            c[3:40] = c[3]                                    # a repeated row
            cols.append(c.to(dtype))
        out.append((cols, torch.randint(0, 2, (B,), generator=g).to(torch.int32)))
    return out


def _init_state(device, N, D, seed):
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for i, f in enumerate(FEATS):
        a = (1.0 / N[i]) ** 0.5
        sd[f"ebc.embedding_bags.t_{f}.weight"] = (torch.rand(N[i], D, generator=g) * 2 - 1) * a
    for tw in ("query_proj", "candidate_proj"):
        k = D
        for l, o in enumerate([128, 64]):
            sd[f"{tw}._mlp.{l}._linear.weight"] = (torch.rand(o, k, generator=g) * 2 - 1) / k ** 0.5
            sd[f"{tw}._mlp.{l}._linear.bias"] = (torch.rand(o, generator=g) * 2 - 1) / k ** 0.5
            k = o
    return {k: v.to(device) for k, v in sd.items()}


@pytest.mark.parametrize("D,dtype", [(128, torch.int64), (64, torch.int32)])
def test_dropin_dispatch_bitwise_equals_fused_ring(device, D, dtype):
    from two_tower_recommender_model_amd.dropin import FusedDropin
    from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

    N, B, lr = [3000, 5000], 256, 0.02
    init = _init_state(device, N, D, seed=D)
    data = _synthetic(N, B, 6, seed=D + 1, dtype=dtype)
    model, opt, pipe = _reference_wiring(device, N, D, lr, lr, init=init)
    it = iter([_kjt_batch(c, l, N, dtype) for c, l in data])
    outs = []
    pipe._model.train()
    while True:
        try:
            loss, logits, labels = pipe.progress(it)
        except StopIteration:
            break
        outs.append((loss.clone(), logits.clone(), labels))
    assert isinstance(pipe._fused, FusedDropin), pipe._fused_reason
    assert pipe._fused.steps_fused == 6 and pipe._fused.steps_generic == 0

    # the same steps on FusedTwoTowerStep's ring directly
    st = FusedTwoTowerStep(N, [D, D], [0], [1], [128, 64], B, device, lr_emb=lr, lr_dense=lr, id_dtype=dtype)
    st.tables.table_view(0).copy_(init["ebc.embedding_bags.t_user_id.weight"])
    st.tables.table_view(1).copy_(init["ebc.embedding_bags.t_product_id.weight"])
    for l in range(2):
        st.qW[l].copy_(init[f"query_proj._mlp.{l}._linear.weight"])
        st.qb[l].copy_(init[f"query_proj._mlp.{l}._linear.bias"])
        st.cW[l].copy_(init[f"candidate_proj._mlp.{l}._linear.weight"])
        st.cb[l].copy_(init[f"candidate_proj._mlp.{l}._linear.bias"])
    st.capture_ring([([c.to(device) for c in cols], lab.to(device)) for cols, lab in data])
    for s in range(len(data)):
        st.run_eager(1)
        torch.cuda.synchronize()
        assert torch.equal(outs[s][1], st.logits), s
        assert torch.equal(outs[s][0], st.loss), s
    sd = model.module.two_tower.state_dict()
    assert torch.equal(sd["ebc.embedding_bags.t_user_id.weight"], st.tables.table_view(0))
    assert torch.equal(sd["ebc.embedding_bags.t_product_id.weight"], st.tables.table_view(1))
    fd = pipe._fused
    assert torch.equal(fd.step.tables.state, st.tables.state)
    for l in range(2):
        assert torch.equal(sd[f"query_proj._mlp.{l}._linear.weight"], st.qW[l])
        assert torch.equal(sd[f"candidate_proj._mlp.{l}._linear.bias"], st.cb[l])
    assert torch.equal(fd.step.exp_avg_sq, st.exp_avg_sq)
    assert int(fd.step.adam_state[0]) == 6
    # the model's parameters ARE the step's buffers (state_dict / eval see the updates)
    w = model.module.two_tower.query_proj._mlp[0]._linear.weight
    assert w.data_ptr() == fd.step.qW[0].data_ptr()


def test_dropin_matches_reference_golden_bf16(device):
    """train_d128 (the reference's TwoTower / TwoTowerTrainTask / transform executed in this container,
    tests/golden/make_golden.py) through the dispatched loop, bf16 tolerances of test_gpu_step.py."""
    from torchrec.datasets.utils import Batch
    from torchrec.sparse.jagged_tensor import KeyedJaggedTensor

    from two_tower_recommender_model_amd.dropin import FusedDropin

    g = load_golden("train_d128.npz")
    D, B, lr = int(g["D"]), int(g["B"]), float(g["lr"])
    N = [int(x) for x in g["num_embeddings"]]
    init = {"ebc.embedding_bags.t_user_id.weight": torch.from_numpy(g["init_t_user_id"]),
            "ebc.embedding_bags.t_product_id.weight": torch.from_numpy(g["init_t_product_id"])}
    for k in g:
        if k.startswith("init_two_tower.") and "proj" in k:
            init[k[len("init_two_tower."):]] = torch.from_numpy(g[k])
    model, opt, pipe = _reference_wiring(device, N, D, lr, lr, layers=[int(x) for x in g["layers"]],
                                         init={k: v.to(device) for k, v in init.items()})

    def batches():
        for s in range(int(g["steps"])):
            kjt = KeyedJaggedTensor.from_lengths_sync(FEATS, torch.from_numpy(g[f"s{s}_values"]),
                                                      torch.from_numpy(np.diff(g[f"s{s}_offsets"]).astype(np.int32)))
            yield Batch(dense_features=torch.zeros(1), sparse_features=kjt,
                        labels=torch.from_numpy(g[f"s{s}_label"]).to(torch.int32))

    it = batches()
    pipe._model.train()
    for s in range(int(g["steps"])):
        loss, logits, _ = pipe.progress(it)
        want = g[f"s{s}_logits"].astype(np.float64)
        err = np.abs(logits.cpu().numpy().astype(np.float64) - want)
        assert np.all(err <= 3e-2 * (np.abs(want).max() + 1e-6) + 1e-5), err.max()
        np.testing.assert_allclose(float(loss), float(g[f"s{s}_loss"]), rtol=1e-2)
    with pytest.raises(StopIteration):
        pipe.progress(it)
    assert isinstance(pipe._fused, FusedDropin) and pipe._fused.steps_fused == int(g["steps"])
    sd = model.module.two_tower.state_dict()

    def check(got, want, atol):
        err = np.abs(got.cpu().numpy() - want)
        assert np.mean(err <= atol) >= 0.99 and err.max() <= 5 * atol, (np.mean(err <= atol), err.max())

    check(sd["ebc.embedding_bags.t_user_id.weight"], g["final_t_user_id"], 5e-3)
    check(sd["ebc.embedding_bags.t_product_id.weight"], g["final_t_product_id"], 5e-3)
    for k in sd:
        if "proj" in k:
            check(sd[k], g["final_two_tower." + k], 3e-2)


def _run_sequence(device, fused_on, monkeypatch):
    """Chunk 1: 4 full batches + a smaller one; chunk 2: 2 full batches; then one eval progress."""
    monkeypatch.setenv("TT_DROPIN_FUSED", "1" if fused_on else "0")
    N, D, B, lr = [2000, 2500], 64, 256, 0.02
    init = _init_state(device, N, D, seed=5)
    model, opt, pipe = _reference_wiring(device, N, D, lr, lr, init=init)
    full = _synthetic(N, B, 7, seed=6)
    part = _synthetic(N, 200, 1, seed=7)[0]
    chunk1 = [_kjt_batch(c, l, N, torch.int64) for c, l in full[:4]] + [_kjt_batch(*part, N, torch.int64)]
    chunk2 = [_kjt_batch(c, l, N, torch.int64) for c, l in full[4:6]]
    losses = []
    pipe._model.train()
    for chunk in (chunk1, chunk2):
        it = iter(chunk)
        while True:
            try:
                loss, _, _ = pipe.progress(it)
            except StopIteration:
                break
            losses.append(float(loss))
    before = model.module.two_tower.state_dict()["ebc.embedding_bags.t_user_id.weight"].clone()
    pipe._model.eval()
    with torch.no_grad():
        eval_loss, eval_logits, _ = pipe.progress(iter([_kjt_batch(*full[6], N, torch.int64)]))
    after = model.module.two_tower.state_dict()["ebc.embedding_bags.t_user_id.weight"]
    assert torch.equal(before, after)
    sd = {k: v.detach().clone() for k, v in model.module.two_tower.state_dict().items()}
    return pipe, losses, float(eval_loss), eval_logits.clone(), sd, opt


def test_dropin_partial_batch_chunks_eval_vs_generic(device, monkeypatch):
    from two_tower_recommender_model_amd.dropin import FusedDropin

    pf, lf, ef, gf, sdf, optf = _run_sequence(device, True, monkeypatch)
    pg, lg, eg, gg, sdg, optg = _run_sequence(device, False, monkeypatch)
    assert isinstance(pf._fused, FusedDropin) and pf._fused.steps_fused == 6 and pf._fused.steps_generic == 1
    assert pg._fused is False
    assert len(lf) == len(lg) == 7
    np.testing.assert_allclose(lf, lg, rtol=1e-2)
    np.testing.assert_allclose(ef, eg, rtol=1e-2)
    # Adam step count carried across the generic batch: 7 steps on every tower parameter, torch's
    # count brought up to date at the chunk's end
    w = pf._model.module.two_tower.query_proj._mlp[0]._linear.weight
    assert int(float(optf._optimizer.state[w]["step"])) == 7
    assert int(pf._fused.step.adam_state[0]) == 7
    for k in sdf:
        a, b = sdf[k].cpu().numpy(), sdg[k].cpu().numpy()
        atol = 5e-3 if "ebc" in k else 3e-2
        err = np.abs(a - b)
        assert np.mean(err <= atol) >= 0.99 and err.max() <= 5 * atol, (k, np.mean(err <= atol), err.max())


def test_dropin_reports_multi_id_bags(device):
    from torchrec.datasets.utils import Batch
    from torchrec.sparse.jagged_tensor import KeyedJaggedTensor

    from two_tower_recommender_model_amd import _lib

    N, D, B = [1000, 1000], 64, 64
    model, opt, pipe = _reference_wiring(device, N, D, 0.01, 0.01)
    good = [_kjt_batch(c, l, N, torch.int64) for c, l in _synthetic(N, B, 2, seed=9)]
    # a batch of 2B ids where one bag holds two ids and another none: the host-side size check passes
    lengths = torch.ones(2 * B, dtype=torch.int32)
    lengths[5], lengths[6] = 2, 0
    bad = Batch(dense_features=torch.zeros(1), labels=torch.zeros(B, dtype=torch.int32),
                sparse_features=KeyedJaggedTensor.from_lengths_sync(FEATS, torch.arange(2 * B) % 1000, lengths))
    pipe._model.train()
    it = iter(good + [bad])
    with pytest.raises(_lib.TTError, match="several ids"):
        while True:
            pipe.progress(it)
