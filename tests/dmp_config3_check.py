"""Child process of tests/test_gpu_dmp.py::test_dmp_config3_shape_world1: BASELINE config 3's shape
(8 single-hot features per tower, 16 tables — user_id 50M rows, product_id 100M rows,
14 side tables of 1M rows — D 128, B 8192, towers [128, 64] over 1024-wide inputs, every table
TABLE_WISE) through DistributedModelParallel -> ShardedEmbeddingBagCollection (HIP backend) ->
TrainPipelineSparseDist over a ONE-rank RCCL group (the 8-GPU plan needs 8 GPUs; this exercises
the shapes, the 16-feature KJT path and the generalised towers on one MI355X).

Oracle on the touched rows only: the ids of the 3 batches are remapped onto compact per-table
copies of the rows they name (read from the GPU shards before training), so the CPU restatement
(`oracle.ref.train_step`) runs on ~1.6e5 rows instead of 1.6e8 with the same arithmetic. Loss and
logits per step rtol 1e-4 (fp32 tower mode), the touched rows after the 3 steps rtol 1e-5 with an
absolute floor of 1e-3 x lr (elements whose gradient cancels), their row-wise Adagrad state rtol
1e-4. Prints DMP-CONFIG3-OK on success.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from child_util import margin, seed_all, stage  # noqa: E402

D, B, LR, LAYERS, STEPS = 128, 8192, 0.05, [128, 64], 3
QUERY = ["user_id"] + [f"u_f{k}" for k in range(1, 8)]
CAND = ["product_id"] + [f"i_f{k}" for k in range(1, 8)]
ROWS = {"user_id": 50_000_000, "product_id": 100_000_000}
ROWS.update({f: 1_000_000 for f in QUERY[1:] + CAND[1:]})


def main():
    device = torch.device("cuda:0")
    torch.cuda.set_device(device)
    seed_all(0)
    stage("init_process_group")
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
    from two_tower_recommender_model_amd.task import TwoTower, TwoTowerTrainTask

    feats = QUERY + CAND  # one table per feature, the EBC's feature (= KeyedTensor) order
    cfgs = [EmbeddingBagConfig(name=f"t_{f}", embedding_dim=D, num_embeddings=ROWS[f], feature_names=[f])
            for f in feats]
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
                                       constraints={c.name: ParameterConstraints(sharding_types=["table_wise"])
                                                    for c in cfgs})
    stage("plan + DMP (allocates ~84 GB of tables)")
    plan = planner.collective_plan(task, get_default_sharders(), dist.group.WORLD)
    model = DistributedModelParallel(module=task, device=device, plan=plan)
    sebc = model.module.two_tower.ebc
    assert isinstance(sebc, ShardedEmbeddingBagCollection)
    assert all(sebc._plan[c.name].sharding_type == "table_wise" for c in cfgs)
    optimizer = KeyedOptimizerWrapper(dict(model.named_parameters()), lambda p: torch.optim.Adam(p, lr=0.01))
    pipeline = TrainPipelineSparseDist(model, optimizer, device)

    stage("batches + compact oracle tables")
    # batches: single-hot, uniform ids in [0, N), ~1 % empty bags
    g = torch.Generator().manual_seed(33)
    host = []
    F = len(feats)
    for _ in range(STEPS + 1):
        lengths = (torch.rand(F * B, generator=g) > 0.01).to(torch.int32)
        vals = []
        for f, name in enumerate(feats):
            n = int(lengths[f * B:(f + 1) * B].sum())
            vals.append(torch.randint(0, ROWS[name], (n,), generator=g))
        host.append((torch.cat(vals), lengths, torch.randint(0, 2, (B,), generator=g).to(torch.int32)))

    # compact oracle tables: the rows the batches touch, read from the GPU shards before training
    def feature_ids(v, lengths, f):
        s = int(lengths[:f * B].sum())
        return v[s:s + int(lengths[f * B:(f + 1) * B].sum())]

    rows = [torch.unique(torch.cat([feature_ids(v, l, f) for v, l, _ in host])) for f in range(F)]
    weights = [sebc.embedding_bags[c.name].weight.detach() for c in cfgs]
    ftab = list(range(F))
    st = ref.TwoTowerState(
        tables=[weights[f][rows[f].to(device)].cpu().clone() for f in range(F)],
        states=[torch.zeros(rows[f].numel()) for f in range(F)], feature_table=ftab,
        query_features=list(range(8)), cand_features=list(range(8, 16)), dims=[D] * F,
        query_layers=[(l._linear.weight.detach().cpu().clone(), l._linear.bias.detach().cpu().clone())
                      for l in model.module.two_tower.query_proj._mlp],
        cand_layers=[(l._linear.weight.detach().cpu().clone(), l._linear.bias.detach().cpu().clone())
                     for l in model.module.two_tower.candidate_proj._mlp])

    def compact(v, lengths):
        out, s = [], 0
        for f in range(F):
            n = int(lengths[f * B:(f + 1) * B].sum())
            out.append(torch.searchsorted(rows[f], v[s:s + n]))
            s += n
        return torch.cat(out)

    def batches(hs):
        for v, l, lab in hs:
            yield Batch(dense_features=torch.zeros(1), sparse_features=KeyedJaggedTensor.from_lengths_sync(feats, v, l),
                        labels=lab)

    it = batches(host[:STEPS])
    pipeline._model.train()
    # margins: max error / allowed error per check (<= 1 passes); printed for every run so the
    # distance from the tolerance is on record, then asserted
    mg = {"loss": 0.0, "logits": 0.0, "rows": 0.0, "state": 0.0}
    for s in range(STEPS):
        stage(f"step {s}")
        loss, logits, _ = pipeline.progress(it)
        v, l, lab = host[s]
        offs = torch.from_numpy(ref.complete_cumsum(l.numpy()))
        want_loss, want_logits, _, _ = ref.train_step(st, compact(v, l), offs, B, lab, LR, 0.01)
        mg["loss"] = max(mg["loss"], margin(float(loss), float(want_loss), 1e-4, 0.0))
        mg["logits"] = max(mg["logits"], margin(logits.cpu().numpy(), want_logits.numpy(), 1e-4, 1e-5))
    torch.cuda.synchronize()
    stage("final rows / states")
    for f, c in enumerate(cfgs):
        got = weights[f][rows[f].to(device)].cpu()
        # an Adagrad step moves an element by lr * G_d / rms(G): where G_d nearly cancels, the GPU
        # and CPU fp32 towers' summation orders (dX rtol ~1e-6) show up at ~3e-4 of the step
        mg["rows"] = max(mg["rows"], margin(got.numpy(), st.tables[f].numpy(), 1e-5, 1e-3 * LR))
        i = sebc._local_index[f]
        got_s = sebc._ts.state_view(i)[rows[f].to(device)].cpu()
        mg["state"] = max(mg["state"], margin(got_s.numpy(), st.states[f].numpy(), 1e-4, 1e-10))
    print("MARGINS " + " ".join(f"{k}={v:.3g}" for k, v in mg.items()), flush=True)
    bad = {k: v for k, v in mg.items() if not v <= 1.0}
    assert not bad, f"outside tolerance (max error / allowed): {bad}"
    del pipeline, model
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print("DMP-CONFIG3-OK", flush=True)
    return 0


if __name__ == "__main__":
    from child_util import child_main

    child_main(main)
