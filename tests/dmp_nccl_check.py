"""Child process of tests/test_gpu_dmp.py (a process group stays out of the pytest process).

The reference's main()/train()/evaluate() wiring (03_model_training.py:770-840, :504-630) on the
torchrec-compatible API over a ONE-rank RCCL ("nccl") process group, so DistributedModelParallel
builds ShardedEmbeddingBagCollection with the HIP lookup backend (as it does at W = 8):

  * 5 tables / 6 multi-hot features (bags of 0..6 ids, empty bags included), a table shared by both
    towers, two tables ROW_WISE and three TABLE_WISE (planner constraints);
  * towers over the concatenation of 3 features each, picked by name from the KeyedTensor
    (torch.cat of kt[f], the reference's pattern 03:420-436, on the HIP KeyedTensor);
  * RowWiseAdagrad in backward (03:791-795), KeyedOptimizerWrapper(Adam) (03:826-829),
    TrainPipelineSparseDist.progress (03:618) for 3 training steps, then eval mode (03:545).

Every step's loss and logits and the final tables (gathered from the ShardedTensor state dict with
the reference's gather_and_get_state_dict, restated from 03:474-495) are compared with the oracle's
train_step (fp32 tower mode: rtol 1e-4 on loss / logits, tables atol 1e-5); eval leaves the tables
unchanged and matches the oracle's forward. Prints DMP-NCCL-OK on success.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

TABLES = [("t_user", 3000, ["user_id"]), ("t_item", 5000, ["product_id"]), ("t_u1", 300, ["u_age"]),
          ("t_shared", 400, ["u_tag", "i_tag"]), ("t_i1", 250, ["i_cat"])]
QUERY = ["user_id", "u_age", "u_tag"]
CAND = ["product_id", "i_tag", "i_cat"]
SHARDING = {"t_user": "row_wise", "t_item": "row_wise", "t_u1": "table_wise", "t_shared": "table_wise",
            "t_i1": "table_wise"}
D, B, LR, LAYERS = 32, 64, 0.05, [64, 32]


def gather_and_get_state_dict(model):
    """03_model_training.py:474-495 (restated): ShardedTensors gathered to rank 0."""
    from torch.distributed._shard.sharded_tensor import ShardedTensor

    rank = dist.get_rank()
    out = {}
    for fqn, tensor in model.state_dict().items():
        if isinstance(tensor, ShardedTensor):
            full = None
            if rank == 0:
                full = torch.zeros(tensor.size()).to(tensor.local_shards()[0].tensor.device)
            tensor.gather(0, full)
            if rank == 0:
                out[fqn] = full
        elif rank == 0:
            out[fqn] = tensor
    return out


def main():
    device = torch.device("cuda:0")
    torch.cuda.set_device(device)
    from child_util import seed_all

    seed_all(0)
    dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(), device_id=device)
    import two_tower_recommender_model_amd as tt
    import two_tower_recommender_model_amd.torchrec.modules.mlp as mlp_mod

    tt.install_torchrec_alias()
    from torch.distributed.optim import _apply_optimizer_in_backward
    from torchrec.datasets.utils import Batch
    from torchrec.distributed import TrainPipelineSparseDist
    from torchrec.distributed.embeddingbag import ShardedEmbeddingBagCollection
    from torchrec.distributed.model_parallel import DistributedModelParallel, get_default_sharders
    from torchrec.distributed.planner import EmbeddingShardingPlanner, ParameterConstraints, Topology
    from torchrec.modules.embedding_configs import EmbeddingBagConfig
    from torchrec.modules.embedding_modules import EmbeddingBagCollection
    from torchrec.optim.keyed import KeyedOptimizerWrapper
    from torchrec.optim.rowwise_adagrad import RowWiseAdagrad
    from torchrec.sparse.jagged_tensor import KeyedJaggedTensor

    from oracle import ref
    from two_tower_recommender_model_amd import ops
    from two_tower_recommender_model_amd.task import TwoTower, TwoTowerTrainTask

    cfgs = [EmbeddingBagConfig(name=n, embedding_dim=D, num_embeddings=r, feature_names=fs) for n, r, fs in TABLES]
    ebc = EmbeddingBagCollection(tables=cfgs, device=torch.device("meta"))
    old = mlp_mod.TOWER_PRECISION
    mlp_mod.TOWER_PRECISION = "fp32"
    try:
        two_tower = TwoTower(ebc, LAYERS, query_features=QUERY, candidate_features=CAND, device=device)
    finally:
        mlp_mod.TOWER_PRECISION = old
    task = TwoTowerTrainTask(two_tower)
    _apply_optimizer_in_backward(RowWiseAdagrad, task.two_tower.ebc.parameters(), {"lr": LR})
    planner = EmbeddingShardingPlanner(topology=Topology(world_size=1, compute_device="cuda"),
                                       constraints={n: ParameterConstraints(sharding_types=[s])
                                                    for n, s in SHARDING.items()})
    plan = planner.collective_plan(task, get_default_sharders(), dist.group.WORLD)
    model = DistributedModelParallel(module=task, device=device, plan=plan)
    sebc = model.module.two_tower.ebc
    assert isinstance(sebc, ShardedEmbeddingBagCollection) and sebc._be is ops.HIP_BACKEND
    assert sorted(sebc._plan[n].sharding_type for n in SHARDING) == sorted(SHARDING.values())
    optimizer = KeyedOptimizerWrapper(dict(model.named_parameters()), lambda p: torch.optim.Adam(p, lr=0.01))
    pipeline = TrainPipelineSparseDist(model, optimizer, device)

    # oracle state: the same initial tables (gathered) and towers
    sd0 = gather_and_get_state_dict(model.module.two_tower)
    keys = [f for _, _, fs in TABLES for f in fs]  # EBC feature order = KeyedTensor order
    ftab = [i for i, (_, _, fs) in enumerate(TABLES) for _ in fs]
    st = ref.TwoTowerState(
        tables=[sd0[f"ebc.embedding_bags.{n}.weight"].cpu().clone() for n, _, _ in TABLES],
        states=[torch.zeros(r) for _, r, _ in TABLES], feature_table=ftab,
        query_features=[keys.index(f) for f in QUERY], cand_features=[keys.index(f) for f in CAND],
        dims=[D] * len(keys),
        query_layers=[(sd0[f"query_proj._mlp.{i}._linear.weight"].cpu().clone(),
                       sd0[f"query_proj._mlp.{i}._linear.bias"].cpu().clone()) for i in range(len(LAYERS))],
        cand_layers=[(sd0[f"candidate_proj._mlp.{i}._linear.weight"].cpu().clone(),
                      sd0[f"candidate_proj._mlp.{i}._linear.bias"].cpu().clone()) for i in range(len(LAYERS))])
    rows = {n: r for n, r, _ in TABLES}
    g = torch.Generator().manual_seed(11)
    host = []
    for s in range(4):
        lengths = torch.randint(0, 7, (len(keys) * B,), generator=g).to(torch.int32)
        lengths[:5] = 0  # empty bags
        vals = [torch.randint(0, rows[TABLES[ftab[i // B]][0]], (int(lengths[i]),), generator=g)
                for i in range(len(keys) * B)]
        host.append((torch.cat(vals).to(torch.int64), lengths, torch.randint(0, 2, (B,), generator=g).to(torch.int32)))

    def batches(hs):
        for v, l, lab in hs:
            yield Batch(dense_features=torch.zeros(1),
                        sparse_features=KeyedJaggedTensor.from_lengths_sync(keys, v, l), labels=lab)

    it = batches(host[:3])
    pipeline._model.train()
    for s in range(3):
        loss, logits, _ = pipeline.progress(it)
        v, l, lab = host[s]
        want_loss, want_logits, _, _ = ref.train_step(st, v, torch.from_numpy(ref.complete_cumsum(l.numpy())), B, lab,
                                                      LR, 0.01)
        np.testing.assert_allclose(float(loss), float(want_loss), rtol=1e-4)
        np.testing.assert_allclose(logits.cpu().numpy(), want_logits.numpy(), rtol=1e-4, atol=1e-5)
    try:
        pipeline.progress(it)
        raise AssertionError("progress() must raise StopIteration on a drained iterator")
    except StopIteration:
        pass
    sd = gather_and_get_state_dict(model.module.two_tower)
    for i, (n, _, _) in enumerate(TABLES):
        np.testing.assert_allclose(sd[f"ebc.embedding_bags.{n}.weight"].cpu().numpy(), st.tables[i].numpy(), rtol=0,
                                   atol=1e-5)
    # eval mode: forward only (03:545); tables untouched
    pipeline._model.eval()
    with torch.no_grad():
        loss, logits, _ = pipeline.progress(batches(host[3:]))
    v, l, lab = host[3]
    pooled = ref.pooled_fwd(st.tables, ftab, v, torch.from_numpy(ref.complete_cumsum(l.numpy())), B)
    q = ref.mlp_fwd(pooled[:, ref.feature_columns(st.dims, st.query_features)], st.query_layers)
    c = ref.mlp_fwd(pooled[:, ref.feature_columns(st.dims, st.cand_features)], st.cand_layers)
    want_logits, want_loss = ref.dot_bce(q, c, lab)
    np.testing.assert_allclose(float(loss), float(want_loss), rtol=1e-4)
    np.testing.assert_allclose(logits.cpu().numpy(), want_logits.numpy(), rtol=1e-4, atol=1e-5)
    sd2 = gather_and_get_state_dict(model.module.two_tower)
    for n, _, _ in TABLES:
        assert torch.equal(sd2[f"ebc.embedding_bags.{n}.weight"], sd[f"ebc.embedding_bags.{n}.weight"])
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print("DMP-NCCL-OK", flush=True)
    return 0


if __name__ == "__main__":
    from child_util import child_main

    child_main(main)
