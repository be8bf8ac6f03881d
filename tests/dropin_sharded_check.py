"""Child of tests/test_gpu_dropin_sharded.py, one process per rank under torch.distributed.run (ranks
share the test box's one MI355X over gloo): the reference's setup and loop (03_model_training.py:
770-829 main(), :612-625 train) at world size W > 1 — DistributedModelParallel ->
ShardedEmbeddingBagCollection -> TrainPipelineSparseDist.progress with KeyedOptimizerWrapper(Adam) —
dispatched to the pipelined fused sharded step (dropin.FusedShardedDropin) on the DMP plan's shards.

--mode bitwise: S fused batches through the loop, then the same S batches on a
FusedShardedTwoTowerStep built directly from the same initial shards, towers and capacity (eager
pipelined steps over the same collectives): per step logits and loss, and at the end every rank's
table shards, row-wise Adagrad state, tower parameters and Adam moments must be BIT-IDENTICAL (the
drop-in is that step on the model's own storage).
--mode mixed: fused batches, a smaller batch (the generic DMP path on every rank), fused batches
again (re-primed), an eval pass: the counts of fused / generic steps, finite losses, and the model's
parameters being the step's buffers.
Prints DROPIN-SHARDED-OK on rank 0."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FEATS = ["user_id", "product_id"]


def make_cols(N, B, rank, step):
    """The raw id columns of (rank, step): some 0 (dropped), some >= N (id % N), some exactly N."""
    g = torch.Generator().manual_seed(7919 * rank + 104729 * step + 5)
    cols = []
    for n in N:
        c = torch.randint(0, 2 * n, (B,), generator=g)
        c[torch.rand(B, generator=g) < 0.05] = 0
        c[:2] = n
        c[2:20] = c[2]
        cols.append(c)
    return cols, torch.randint(0, 2, (B,), generator=g).to(torch.int32)


def kjt_batch(cols, labels, N, device):
    """transform_to_torchrec_batch (03:353-380), vectorised: id 0 dropped, id % N kept."""
    from torchrec.datasets.utils import Batch
    from torchrec.sparse.jagged_tensor import KeyedJaggedTensor

    vals, lens = [], []
    for c, n in zip(cols, N):
        keep = c != 0
        vals.append(torch.remainder(c[keep], n))
        lens.append(keep.to(torch.int32))
    kjt = KeyedJaggedTensor.from_lengths_sync(FEATS, torch.cat(vals), torch.cat(lens))
    return Batch(dense_features=torch.zeros(1), sparse_features=kjt, labels=labels).to(device)


def main():
    from child_util import stage

    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="bitwise", choices=["bitwise", "mixed"])
    ap.add_argument("--plan", default="default", choices=["default", "tw", "mixed"])
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--dim", type=int, default=128)
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    device = torch.device("cuda:0")  # every rank on the box's one GPU (the rehearsal)
    torch.cuda.set_device(device)
    dist.init_process_group("gloo")
    import two_tower_recommender_model_amd as tt

    tt.install_torchrec_alias()
    from torch.distributed.optim import _apply_optimizer_in_backward
    from torchrec.distributed import TrainPipelineSparseDist
    from torchrec.distributed.model_parallel import DistributedModelParallel, get_default_sharders
    from torchrec.distributed.planner import EmbeddingShardingPlanner, ParameterConstraints, Topology
    from torchrec.modules.embedding_configs import EmbeddingBagConfig
    from torchrec.modules.embedding_modules import EmbeddingBagCollection
    from torchrec.optim.keyed import KeyedOptimizerWrapper
    from torchrec.optim.rowwise_adagrad import RowWiseAdagrad

    from two_tower_recommender_model_amd.dropin import FusedShardedDropin
    from two_tower_recommender_model_amd.sharded import FusedShardedTwoTowerStep, TorchComm
    from two_tower_recommender_model_amd.task import TwoTower, TwoTowerTrainTask

    N, D, B, S, lr = [30_000, 50_000], args.dim, args.batch, args.steps, 0.02
    torch.manual_seed(11)
    stage("wiring")
    cfgs = [EmbeddingBagConfig(name=f"t_{f}", embedding_dim=D, num_embeddings=N[i], feature_names=[f])
            for i, f in enumerate(FEATS)]
    ebc = EmbeddingBagCollection(tables=cfgs, device=torch.device("meta"))
    task = TwoTowerTrainTask(TwoTower(embedding_bag_collection=ebc, layer_sizes=[128, 64], device=device))
    _apply_optimizer_in_backward(RowWiseAdagrad, task.two_tower.ebc.parameters(), {"lr": lr})
    cons = {"default": {}, "tw": {"t_user_id": "table_wise", "t_product_id": "table_wise"},
            "mixed": {"t_user_id": "table_wise", "t_product_id": "row_wise"}}[args.plan]
    planner = EmbeddingShardingPlanner(topology=Topology(world_size=world, compute_device="cuda"),
                                       constraints={k: ParameterConstraints(sharding_types=[v]) for k, v in cons.items()})
    plan = planner.collective_plan(task, get_default_sharders(), dist.group.WORLD) if cons else None
    model = DistributedModelParallel(module=task, device=device, plan=plan)
    opt = KeyedOptimizerWrapper(dict(model.named_parameters()), lambda ps: torch.optim.Adam(ps, lr=lr))
    pipe = TrainPipelineSparseDist(model, opt, device)
    sebc = model.module.two_tower.ebc
    towers = [model.module.two_tower.query_proj, model.module.two_tower.candidate_proj]
    tparams = [p for tw_ in towers for l in tw_._mlp for p in (l._linear.weight, l._linear.bias)]
    # initial state (identical towers on every rank after DDP's broadcast; this rank's shards)
    init_local = {t: sebc._ts.table_view(i)[:n].clone() for (t, lo, n), i in
                  zip(sebc._local_tables, range(len(sebc._local_tables)))} if sebc._ts is not None else {}
    init_towers = torch.cat([p.detach().reshape(-1).clone() for p in tparams])
    data = [make_cols(N, B, rank, s) for s in range(S)]
    pipe._model.train()
    stage("drop-in loop")
    outs = []
    if args.mode == "bitwise":
        it = iter([kjt_batch(c, l, N, device) for c, l in data])
        while True:
            try:
                loss, logits, _ = pipe.progress(it)
            except StopIteration:
                break
            outs.append((loss.clone(), logits.clone()))
        fd = pipe._fused
        assert isinstance(fd, FusedShardedDropin), pipe._fused_reason
        assert fd.steps_fused == S and fd.steps_generic == 0, (fd.steps_fused, fd.steps_generic)
        print(f"rank {rank}: dispatch {pipe._fused_reason}, sharding {fd.sharding} owners {fd.owners}, "
              f"capacity {fd.step.caps_f}, graphs {fd.graph_mode}", flush=True)
        # the same steps on the sharded step built directly
        stage("direct step")
        ref = FusedShardedTwoTowerStep(TorchComm(always_collective=True), N, D, [128, 64], B, device,
                                       sharding=fd.sharding, tw_owners=fd.owners, lr_emb=lr, lr_dense=lr,
                                       capacity=list(fd.step.caps_f))
        for f in range(2):
            li = sebc._local_index.get(sebc._f_table[f])
            if li is not None:
                n = ref.local_rows[f]
                ref.tables.table_view(f)[:n].copy_(init_local[sebc._f_table[f]])
        ref.params.copy_(init_towers)
        ref.towers.update(ref.params, do_adam=False)
        pool = []
        for cols, lab in data:
            cc = []
            for c, n in zip(cols, N):
                v = torch.remainder(c, n)
                cc.append(torch.where(c == 0, 0, torch.where(v == 0, n, v)).to(device))
            pool.append((cc, lab.to(device)))
        ref.prime(pool[0][0], 0, pool[1][0])
        ref.cursor = 0
        zero = [torch.zeros(B, dtype=torch.int64, device=device) for _ in range(2)]
        for s in range(S):
            ref.step_pipelined(pool[s][1], s % 2, pool[s + 2][0] if s + 2 < S else zero)
            torch.cuda.synchronize()
            assert torch.equal(outs[s][1], ref.logits), f"rank {rank} step {s}: logits differ"
            assert torch.equal(outs[s][0], ref.loss), f"rank {rank} step {s}: loss differs"
        st = fd.step
        for f in range(2):
            assert torch.equal(st.tables.table_view(f), ref.tables.table_view(f)[:ref.local_rows[f]]), f"table {f}"
            assert torch.equal(st.tables.state_view(f), ref.tables.state_view(f)[:ref.local_rows[f]]), f"state {f}"
        assert torch.equal(st.params, ref.params) and torch.equal(st.exp_avg, ref.exp_avg)
        assert torch.equal(st.exp_avg_sq, ref.exp_avg_sq)
        assert int(st.adam_state[0]) == S
        # the model's parameters and shards ARE the step's storage
        assert tparams[0].data_ptr() == st.params.data_ptr()
        if sebc._ts is not None:
            assert st.tables.weights.data_ptr() == sebc._ts.weights.data_ptr()
        del ref
    else:
        half = make_cols(N, B // 2, rank, 99)
        seq = [kjt_batch(c, l, N, device) for c, l in data[:S // 2]] + [kjt_batch(*half, N, device)] + \
              [kjt_batch(c, l, N, device) for c, l in data[S // 2:]]
        it = iter(seq)
        n = 0
        while True:
            try:
                loss, logits, _ = pipe.progress(it)
            except StopIteration:
                break
            assert torch.isfinite(loss).all(), f"step {n}: loss {float(loss)}"
            n += 1
        fd = pipe._fused
        assert isinstance(fd, FusedShardedDropin), pipe._fused_reason
        assert fd.steps_fused == S and fd.steps_generic == 1, (fd.steps_fused, fd.steps_generic)
        # eval: forward-only through the generic path on the trained storage
        pipe._model.eval()
        with torch.no_grad():
            ev = iter([kjt_batch(c, l, N, device) for c, l in data[:2]])
            for _ in range(2):
                loss, logits, _ = pipe.progress(ev)
                assert torch.isfinite(loss).all()
        assert tparams[0].data_ptr() == fd.step.params.data_ptr()
    torch.cuda.synchronize()
    del pipe, model, opt
    dist.barrier()
    if rank == 0:
        print("DROPIN-SHARDED-OK", flush=True)
    return 0


if __name__ == "__main__":
    from child_util import child_main

    child_main(main)
