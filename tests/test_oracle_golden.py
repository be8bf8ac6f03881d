"""Pin the oracle: the CPU restatement (oracle/ref.py) against golden vectors produced by executing
the reference's own transform_to_torchrec_batch / TwoTower / TwoTowerTrainTask code
(tests/golden/make_golden.py). CPU only."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import ref


@pytest.mark.parametrize("case", ["i32", "i64", "big", "allzero"])
def test_kjt_build_matches_reference_transform(case):
    g = load_golden(f"kjt_{case}.npz")
    values, lengths, offsets = ref.kjt_build([g["user_id"], g["product_id"]], list(g["num_embeddings"]))
    assert values.dtype == g["values"].dtype, (values.dtype, g["values"].dtype)
    np.testing.assert_array_equal(values, g["values"])
    np.testing.assert_array_equal(lengths, g["lengths"])
    np.testing.assert_array_equal(offsets, g["offsets"])
    assert g["labels_out"].dtype == np.int32


def _state_from_golden(g):
    layers = [int(x) for x in g["layers"]]
    D = int(g["D"])
    st = ref.TwoTowerState(
        tables=[torch.from_numpy(g["init_t_user_id"]).clone(), torch.from_numpy(g["init_t_product_id"]).clone()],
        states=[torch.zeros(int(n)) for n in g["num_embeddings"]],
        feature_table=[0, 1], query_features=[0], cand_features=[1], dims=[D, D],
        query_layers=[(torch.from_numpy(g[f"init_two_tower.query_proj._mlp.{i}._linear.weight"]).clone(),
                       torch.from_numpy(g[f"init_two_tower.query_proj._mlp.{i}._linear.bias"]).clone())
                      for i in range(len(layers))],
        cand_layers=[(torch.from_numpy(g[f"init_two_tower.candidate_proj._mlp.{i}._linear.weight"]).clone(),
                      torch.from_numpy(g[f"init_two_tower.candidate_proj._mlp.{i}._linear.bias"]).clone())
                     for i in range(len(layers))],
    )
    return st, layers


@pytest.mark.parametrize("case", ["c1", "c1full", "zipf", "d128"])
@pytest.mark.parametrize("sparse_update", [True, False])
def test_train_step_matches_reference_task(case, sparse_update):
    g = load_golden(f"train_{case}.npz")
    st, layers = _state_from_golden(g)
    B = int(g["B"])
    lr = float(g["lr"])
    for s in range(int(g["steps"])):
        values, lengths, offsets = ref.kjt_build([g[f"s{s}_user_id"], g[f"s{s}_product_id"]], list(g["num_embeddings"]))
        np.testing.assert_array_equal(values, g[f"s{s}_values"])
        loss, logits, pooled, gpooled = ref.train_step(
            st, torch.from_numpy(values), torch.from_numpy(offsets), B, torch.from_numpy(g[f"s{s}_label"]),
            lr_emb=lr, lr_dense=lr, sparse_update=sparse_update)
        np.testing.assert_allclose(pooled.numpy(), g[f"s{s}_pooled"], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(logits.numpy(), g[f"s{s}_logits"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(float(loss), float(g[f"s{s}_loss"]), rtol=1e-6)
        np.testing.assert_allclose(gpooled.numpy(), g[f"s{s}_pooled_grad"], rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(st.tables[0].numpy(), g["final_t_user_id"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(st.tables[1].numpy(), g["final_t_product_id"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(st.states[0].numpy(), g["final_state_t_user_id"], rtol=1e-5, atol=1e-12)
    np.testing.assert_allclose(st.states[1].numpy(), g["final_state_t_product_id"], rtol=1e-5, atol=1e-12)
    for i in range(len(layers)):
        np.testing.assert_allclose(st.query_layers[i][0].numpy(),
                                   g[f"final_two_tower.query_proj._mlp.{i}._linear.weight"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(st.cand_layers[i][1].numpy(),
                                   g[f"final_two_tower.candidate_proj._mlp.{i}._linear.bias"], rtol=1e-5, atol=1e-6)


def test_complete_cumsum_and_permute_roundtrip():
    rng = np.random.default_rng(0)
    F_, B = 5, 17
    lengths = rng.integers(0, 4, F_ * B).astype(np.int32)
    values = rng.integers(0, 1000, int(lengths.sum())).astype(np.int64)
    perm = [3, 1, 4, 0, 2]
    l2, v2, _ = ref.kjt_permute(lengths, values, F_, B, perm)
    inv = [perm.index(i) for i in range(F_)]
    l3, v3, _ = ref.kjt_permute(l2, v2, F_, B, inv)
    np.testing.assert_array_equal(l3, lengths)
    np.testing.assert_array_equal(v3, values)


def test_block_bucketize_reassembles():
    rng = np.random.default_rng(1)
    F_, B, W = 2, 9, 3
    N = [10, 25]
    lengths = rng.integers(0, 4, F_ * B).astype(np.int32)
    vals = []
    offs = ref.complete_cumsum(lengths)
    for i in range(F_ * B):
        vals.extend(rng.integers(0, N[i // B] + 5, lengths[i]).tolist())  # some ids beyond bs*W
    values = np.asarray(vals, np.int64)
    bs = [(n + W - 1) // W for n in N]
    nl, nv = ref.block_bucketize(lengths, values, F_, B, bs, W)
    assert nl.size == W * F_ * B and nv.size == values.size
    no = ref.complete_cumsum(nl)
    # exact inverse: in-block ids have local < bs (id = p*bs + local); ids >= bs*W have
    # local = id // W >= bs (id = local*W + p)
    for i in range(F_ * B):
        f = i // B
        got = []
        for p in range(W):
            k = p * F_ * B + i
            for loc in nv[no[k]:no[k + 1]]:
                loc = int(loc)
                got.append(p * bs[f] + loc if loc < bs[f] else loc * W + p)
        assert sorted(got) == sorted(values[offs[i]:offs[i + 1]].tolist())


def test_batch_of_one_raises_like_the_reference():
    """03_model_training.py:452 squeezes the logits of a batch of one to 0-d; BCEWithLogitsLoss then
    rejects the [1] labels. The oracle keeps that behaviour (the drop-in task raises the same)."""
    import pytest
    import torch

    from oracle import ref

    with pytest.raises(ValueError, match="must be the same as input size"):
        ref.dot_bce(torch.rand(1, 4), torch.rand(1, 4), torch.ones(1))
