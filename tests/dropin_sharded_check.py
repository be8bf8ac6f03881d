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
again (re-primed), an eval pass: the counts of fused / generic steps, finite losses, the model's
parameters being the step's buffers, and the whole run against the same batches through the
generic DMP path alone (TT_DROPIN_FUSED=0, a second model from the same initial state): per-step
losses, every rank's shards and the towers within the bf16 towers' tolerance.
--mode skew: a later batch whose ids all fall in rank 0's row block (past the capacity the first
batch sized) and one batch with a bag of two ids: the agreed admission sends both down the generic
path on every rank (nothing raises at StopIteration, no fused step trains on dropped lookups), and
the run equals the generic-only run as in mixed.
--mode kjt: multi-hot bags from the first batch (BASELINE config 5's shape, scaled down): the
drop-in's kjt mode (sharded_kjt.FusedShardedKJTStep) bit for bit against that step built directly
(eager, TorchComm) on the same shards, towers, capacity and batches.
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


def make_multihot(N, B, rank, step, maxlen=5):
    """Bags of 1..maxlen ids in range (key-major values, lengths) for (rank, step)."""
    g = torch.Generator().manual_seed(1299709 * rank + 15485863 * step + 3)
    vals, lens = [], []
    for n in N:
        ln = torch.randint(1, maxlen + 1, (B,), generator=g, dtype=torch.int32)
        ln[torch.rand(B, generator=g) < 0.05] = 0  # some empty bags
        vals.append(torch.randint(0, n, (int(ln.sum()),), generator=g))
        lens.append(ln)
    return torch.cat(vals), torch.cat(lens), torch.randint(0, 2, (B,), generator=g).to(torch.int32)


def kjt_multihot_batch(vals, lens, labels, device):
    from torchrec.datasets.utils import Batch
    from torchrec.sparse.jagged_tensor import KeyedJaggedTensor

    kjt = KeyedJaggedTensor.from_lengths_sync(FEATS, vals, lens)
    return Batch(dense_features=torch.zeros(1), sparse_features=kjt, labels=labels).to(device)


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


def build(args, world, device, lr):
    """The reference's wiring (03_model_training.py:770-829): EBC on meta, TwoTower, task,
    in-backward RowWiseAdagrad, DMP (the plan), KeyedOptimizerWrapper(Adam), the pipeline."""
    from torch.distributed.optim import _apply_optimizer_in_backward
    from torchrec.distributed import TrainPipelineSparseDist
    from torchrec.distributed.model_parallel import DistributedModelParallel, get_default_sharders
    from torchrec.distributed.planner import EmbeddingShardingPlanner, ParameterConstraints, Topology
    from torchrec.modules.embedding_configs import EmbeddingBagConfig
    from torchrec.modules.embedding_modules import EmbeddingBagCollection
    from torchrec.optim.keyed import KeyedOptimizerWrapper
    from torchrec.optim.rowwise_adagrad import RowWiseAdagrad

    from two_tower_recommender_model_amd.task import TwoTower, TwoTowerTrainTask

    N, D = args.N, args.dim
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
    return model, opt, pipe, sebc, tparams


def run_loop(pipe, batches):
    pipe._model.train()
    it = iter(batches)
    outs = []
    while True:
        try:
            loss, logits, _ = pipe.progress(it)
        except StopIteration:
            break
        outs.append((loss.detach().clone(), logits.detach().clone()))
    torch.cuda.synchronize()
    return outs


def compare_with_generic(args, world, rank, device, lr, batches, a, outs_a):
    """A second model from A's initial state, the same batches through the generic DMP path only
    (TT_DROPIN_FUSED=0): per-step losses, this rank's shards and the towers within the bf16 towers'
    tolerance (the fused and per-op towers round at different points)."""
    model_a, sebc_a, tparams_a, init = a
    model_b, opt_b, pipe_b, sebc_b, tparams_b = build(args, world, device, lr)
    with torch.no_grad():
        if sebc_b._ts is not None:
            sebc_b._ts.weights.copy_(init["weights"])
            sebc_b._ts.state.zero_()
        for p, v in zip(tparams_b, init["towers"]):
            p.copy_(v)
    os.environ["TT_DROPIN_FUSED"] = "0"
    try:
        outs_b = run_loop(pipe_b, batches)
    finally:
        os.environ.pop("TT_DROPIN_FUSED", None)
    assert pipe_b._fused is False, pipe_b._fused_reason
    assert len(outs_a) == len(outs_b), (len(outs_a), len(outs_b))
    worst = {"loss": 0.0, "rows": 0.0, "towers": 0.0}
    for s, ((la, _), (lb, _)) in enumerate(zip(outs_a, outs_b)):
        d = abs(float(la) - float(lb))
        worst["loss"] = max(worst["loss"], d)
        assert d <= 2e-3 * max(1.0, abs(float(lb))), f"rank {rank} step {s}: loss {float(la)} vs {float(lb)}"
    if sebc_a._ts is not None:
        wa, wb = sebc_a._ts.weights, sebc_b._ts.weights
        w0 = init["weights"]
        da, db = wa - w0, wb - w0  # the updates (rows untouched by both: exactly 0)
        D = args.dim
        # every lookup reached its row in both runs: the same rows moved (a dropped lookup would
        # leave its row untouched in one of them)
        ta, tb = (da.view(-1, D) != 0).any(dim=-1), (db.view(-1, D) != 0).any(dim=-1)
        assert torch.equal(ta, tb), f"rank {rank}: touched rows differ ({int((ta != tb).sum())} rows)"
        e = (da - db).abs().view(-1, D)[tb]
        scale = db.abs().max().item()
        q = torch.quantile(e.flatten().float()[:1 << 24], torch.tensor([0.5, 0.99, 0.999], device=e.device)).tolist()
        err = e.max().item()
        worst["rows"] = err / max(scale, 1e-30)
        print(f"rank {rank}: row updates |fused - generic| p50 {q[0]:.3g} p99 {q[1]:.3g} p99.9 {q[2]:.3g} max {err:.3g} "
              f"(largest update {scale:.3g}, {int(tb.sum())} rows)", flush=True)
        # the towers round at different points (fused bf16 MFMA chain vs per-op bf16 GEMMs), and the
        # row-wise Adagrad normalises each row's gradient: a row whose gradient nearly cancels (a
        # hot row summed over many lookups) moves by a noisy direction in both. Bulk bound + a
        # loose bound on the worst element
        assert q[1] <= 2e-2 * scale and q[2] <= 5e-2 * scale and err <= 0.25 * scale, \
            f"rank {rank}: shard updates differ (p99 {q[1]}, p99.9 {q[2]}, max {err}; largest {scale})"
    # towers: Adam normalises every element's step (m / sqrt(v): about +-lr at the first steps), so an
    # element whose gradient is near zero may step either way in the two runs (at most 2 lr per
    # step apart); the bulk must agree: compare the parameters' updates by quantiles
    ua = torch.cat([(p.detach() - v).flatten() for p, v in zip(tparams_a, init["towers"])])
    ub = torch.cat([(q.detach() - v).flatten() for q, v in zip(tparams_b, init["towers"])])
    e = (ua - ub).abs()
    q = torch.quantile(e.float(), torch.tensor([0.5, 0.9, 0.99], device=e.device)).tolist()
    scale = ub.abs().max().item()
    worst["towers"] = q[2] / max(scale, 1e-30)
    print(f"rank {rank}: tower updates |fused - generic| p50 {q[0]:.3g} p90 {q[1]:.3g} p99 {q[2]:.3g} max "
          f"{e.max().item():.3g} (largest update {scale:.3g})", flush=True)
    steps = len(outs_a)
    assert q[0] <= 2e-2 * scale and q[1] <= 1e-1 * scale and e.max().item() <= 2 * lr * steps + 1e-6, \
        f"rank {rank}: tower updates differ (p50 {q[0]}, p90 {q[1]}, max {e.max().item()}; largest {scale})"
    print(f"rank {rank}: fused dispatch vs generic-only run, worst relative: {worst}", flush=True)
    del model_b, opt_b, pipe_b


def main():
    from child_util import stage

    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="bitwise", choices=["bitwise", "mixed", "skew", "kjt"])
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
    from two_tower_recommender_model_amd.dropin import FusedShardedDropin
    from two_tower_recommender_model_amd.sharded import FusedShardedTwoTowerStep, TorchComm
    from two_tower_recommender_model_amd.sharded_kjt import FusedShardedKJTStep

    N, D, B, S, lr = [30_000, 50_000], args.dim, args.batch, args.steps, 0.02
    args.N = N
    torch.manual_seed(11)
    stage("wiring")
    model, opt, pipe, sebc, tparams = build(args, world, device, lr)
    # initial state (identical towers on every rank after DDP's broadcast; this rank's shards)
    init_local = {t: sebc._ts.table_view(i)[:n].clone() for (t, lo, n), i in
                  zip(sebc._local_tables, range(len(sebc._local_tables)))} if sebc._ts is not None else {}
    init = {"weights": sebc._ts.weights.clone() if sebc._ts is not None else None,
            "towers": [p.detach().clone() for p in tparams]}
    init_towers = torch.cat([p.detach().reshape(-1).clone() for p in tparams])
    data = [make_cols(N, B, rank, s) for s in range(S)]
    stage("drop-in loop")
    if args.mode == "bitwise":
        outs = run_loop(pipe, [kjt_batch(c, l, N, device) for c, l in data])
        fd = pipe._fused
        assert isinstance(fd, FusedShardedDropin), pipe._fused_reason
        assert fd.mode == "pipelined" and fd.steps_fused == S and fd.steps_generic == 0, \
            (fd.mode, fd.steps_fused, fd.steps_generic, fd.rejected)
        print(f"rank {rank}: dispatch {pipe._fused_reason}, sharding {fd.sharding} owners {fd.owners}, "
              f"capacity {fd.step.caps_f}, graphs {fd.graph_mode}, exchange {fd.exchange}", flush=True)
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
            n = ref.local_rows[f]
            assert torch.equal(st.tables.table_view(f)[:n], ref.tables.table_view(f)[:n]), f"table {f}"
            assert torch.equal(st.tables.state_view(f)[:n], ref.tables.state_view(f)[:n]), f"state {f}"
        assert torch.equal(st.params, ref.params) and torch.equal(st.exp_avg, ref.exp_avg)
        assert torch.equal(st.exp_avg_sq, ref.exp_avg_sq)
        assert int(st.adam_state[0]) == S
        # the model's parameters and shards ARE the step's storage
        assert tparams[0].data_ptr() == st.params.data_ptr()
        if sebc._ts is not None:
            assert st.tables.weights.data_ptr() == sebc._ts.weights.data_ptr()
        del ref
    elif args.mode == "kjt":
        mh = [make_multihot(N, B, rank, s) for s in range(S)]
        outs = run_loop(pipe, [kjt_multihot_batch(v, ln, lab, device) for v, ln, lab in mh])
        fd = pipe._fused
        assert isinstance(fd, FusedShardedDropin), pipe._fused_reason
        assert fd.mode == "kjt" and fd.steps_fused == S and fd.steps_generic == 0, \
            (fd.mode, fd.steps_fused, fd.steps_generic, fd.rejected)
        print(f"rank {rank}: kjt mode, sharding {fd.sharding} owners {fd.owners}, cap {fd.step.cap}, graphs "
              f"{fd.graph_mode}, exchange {fd.exchange}", flush=True)
        stage("direct KJT step")
        ref = FusedShardedKJTStep(TorchComm(always_collective=True), N, D, [128, 64], B, device, fd.step.cap,
                                  sharding=fd.sharding, tw_owners=fd.owners, lr_emb=lr, lr_dense=lr)
        for f in range(2):
            li = sebc._local_index.get(sebc._f_table[f])
            if li is not None:
                n = ref.local_rows[f]
                ref.tables.table_view(f)[:n].copy_(init_local[sebc._f_table[f]])
        ref.params.copy_(init_towers)
        ref.towers.update(ref.params, do_adam=False)
        ref.warmup()
        for s, (v, ln, lab) in enumerate(mh):
            o = torch.zeros(ln.numel() + 1, dtype=torch.int32)
            o[1:] = torch.cumsum(ln, 0)
            ref.step(v.to(device), o.to(device), lab.to(device))
            torch.cuda.synchronize()
            assert torch.equal(outs[s][1], ref.logits), f"rank {rank} step {s}: logits differ"
            assert torch.equal(outs[s][0], ref.loss), f"rank {rank} step {s}: loss differs"
        st = fd.step
        for f in range(2):
            n = ref.local_rows[f]
            assert torch.equal(st.tables.table_view(f)[:n], ref.tables.table_view(f)[:n]), f"table {f}"
            assert torch.equal(st.tables.state_view(f)[:n], ref.tables.state_view(f)[:n]), f"state {f}"
        assert torch.equal(st.params, ref.params) and torch.equal(st.exp_avg, ref.exp_avg)
        assert torch.equal(st.exp_avg_sq, ref.exp_avg_sq)
        assert tparams[0].data_ptr() == st.params.data_ptr()
        del ref
        # and the whole run against the generic DMP path on the same batches
        stage("generic-only run (kjt)")
        compare_with_generic(args, world, rank, device, lr, [kjt_multihot_batch(v, ln, lab, device) for v, ln, lab in mh],
                             (model, sebc, tparams, init), outs)
    else:
        if args.mode == "mixed":
            half = make_cols(N, B // 2, rank, 99)
            seq = [kjt_batch(c, l, N, device) for c, l in data[:S // 2]] + [kjt_batch(*half, N, device)] + \
                  [kjt_batch(c, l, N, device) for c, l in data[S // 2:]]
            n_generic, why = 1, None
        else:  # skew: batch S//2 has every item id in rank 0's row block; batch S//2 + 2 a two-id bag
            cols, lab = make_cols(N, B, rank, 77)
            cols[1] = torch.remainder(cols[1], N[1] // world)
            cols[1][cols[1] == 0] = 1
            seq = [kjt_batch(c, l, N, device) for c, l in data]
            seq.insert(S // 2, kjt_batch(cols, lab, N, device))
            mv, ml, mlab = make_multihot(N, B, rank, 5, maxlen=1)
            ml[3] = 2 if rank == world - 1 else 1  # only the last rank has a bag of two ids
            mv = torch.randint(1, N[0], (int(ml.sum()),))
            seq.insert(S // 2 + 2, kjt_multihot_batch(mv, ml, mlab, device))
            n_generic = 2
        outs = run_loop(pipe, seq)
        fd = pipe._fused
        assert isinstance(fd, FusedShardedDropin), pipe._fused_reason
        assert all(torch.isfinite(l).all() for l, _ in outs)
        assert fd.steps_fused == S and fd.steps_generic == n_generic, \
            (fd.steps_fused, fd.steps_generic, fd.rejected)
        print(f"rank {rank}: {args.mode}: fused {fd.steps_fused}, generic {fd.steps_generic}, rejected {fd.rejected}, "
              f"capacity {fd.step.caps_f}, exchange {fd.exchange}", flush=True)
        if args.mode == "skew":
            assert any("capacity" in k for k in fd.rejected), fd.rejected
            assert any("several ids" in k for k in fd.rejected), fd.rejected
        assert tparams[0].data_ptr() == fd.step.params.data_ptr()
        stage("generic-only run")
        compare_with_generic(args, world, rank, device, lr, seq, (model, sebc, tparams, init), outs)
        if args.mode == "mixed":
            # eval: forward-only through the generic path on the trained storage
            pipe._model.eval()
            with torch.no_grad():
                ev = iter([kjt_batch(c, l, N, device) for c, l in data[:2]])
                for _ in range(2):
                    loss, logits, _ = pipe.progress(ev)
                    assert torch.isfinite(loss).all()
    torch.cuda.synchronize()
    del pipe, model, opt
    dist.barrier()
    if rank == 0:
        print("DROPIN-SHARDED-OK", flush=True)
    return 0


if __name__ == "__main__":
    from child_util import child_main

    child_main(main)
