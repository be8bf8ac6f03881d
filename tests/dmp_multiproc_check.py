"""Child of tests/test_gpu_dmp_multiproc.py, one process per rank under torch.distributed.run: the
reference's setup and loop (03_model_training.py:770-829 main(), :612-625 train) through
DistributedModelParallel -> ShardedEmbeddingBagCollection (the HIP lookup backend) ->
TrainPipelineSparseDist with KeyedOptimizerWrapper(Adam) and bf16 MFMA towers, at BASELINE.json's
table sizes, W ranks sharing the one GPU of the test box over a gloo process group (the production
run is RCCL, one GPU per rank: eight processes on one MI355X is the rehearsal of that run):

  config3  16 single-hot tables (user_id 50M, product_id 100M, 14 x 1M rows), 8 features per tower,
           every table TABLE_WISE, D 128 (84 GB of tables over the ranks)
  config5  user_id 50M rows TABLE_WISE, product_id 100M rows ROW_WISE (mixed TW + RW), multi-hot
           bags of Uniform{1..39} ids (mean 20), D 128

The oracle runs on rank 0 on the TOUCHED rows only: every rank's batches are seeded by (rank,
step), so every process knows all of them; before every step the owners send the touched rows of
their shards (and row-wise Adagrad state) to rank 0, with the towers and their Adam moments. Per
step and rank, against that state: the pooled rows (torch CPU embedding_bag sums of the compact
rows), the bf16 towers' logits element-wise against tower_emul (its bounds carrying the fp32
summation-order error of the pooled sums), the loss; then every touched row's update against
oracle.ref's RowWiseAdagrad fed the SUM over ranks of the emulated pooled gradients
(tower_emul.check_adagrad, TorchRec's sharded EBC semantics), and the towers against Adam on the
MEAN over ranks of the emulated tower gradients (DDP; tower_emul.check_adam). Prints
DMP-MULTIPROC-OK on rank 0."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

D, LR, LAYERS = 128, 0.01, [128, 64]
QUERY3 = ["user_id"] + [f"u_f{k}" for k in range(1, 8)]
CAND3 = ["product_id"] + [f"i_f{k}" for k in range(1, 8)]


def workload(name):
    if name == "config3":
        rows = {"user_id": 50_000_000, "product_id": 100_000_000}
        rows.update({f: 1_000_000 for f in QUERY3[1:] + CAND3[1:]})
        feats = QUERY3 + CAND3
        return dict(feats=feats, rows=rows, query=QUERY3, cand=CAND3, maxlen=0,
                    sharding={f: "table_wise" for f in feats})
    if name == "config5":
        return dict(feats=["user_id", "product_id"], rows={"user_id": 50_000_000, "product_id": 100_000_000},
                    query=["user_id"], cand=["product_id"], maxlen=39,
                    sharding={"user_id": "table_wise", "product_id": "row_wise"})
    raise SystemExit(f"unknown workload {name}")


def make_batch(wl, B, rank, step):
    """(values int64, lengths int32 [F*B], labels int32 [B]) of (rank, step), key-major."""
    g = torch.Generator().manual_seed(7919 * rank + 104729 * step + 17)
    F = len(wl["feats"])
    if wl["maxlen"]:
        lengths = torch.randint(1, wl["maxlen"] + 1, (F * B,), generator=g).to(torch.int32)
    else:
        lengths = (torch.rand(F * B, generator=g) > 0.01).to(torch.int32)  # ~1 % empty bags
    vals = [torch.randint(0, wl["rows"][f], (int(lengths[i * B:(i + 1) * B].sum()),), generator=g)
            for i, f in enumerate(wl["feats"])]
    return torch.cat(vals), lengths, torch.randint(0, 2, (B,), generator=g).to(torch.int32)


def feature_ids(v, lengths, i, B):
    s = int(lengths[:i * B].sum())
    return v[s:s + int(lengths[i * B:(i + 1) * B].sum())]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", required=True)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    device = torch.device("cuda:0")  # every rank on the box's one GPU (the rehearsal)
    torch.cuda.set_device(device)
    dist.init_process_group("gloo")
    import two_tower_recommender_model_amd as tt

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

    from two_tower_recommender_model_amd.task import TwoTower, TwoTowerTrainTask

    wl = workload(args.workload)
    B, S, feats = args.batch, args.steps, wl["feats"]
    F = len(feats)
    cfgs = [EmbeddingBagConfig(name=f"t_{f}", embedding_dim=D, num_embeddings=wl["rows"][f], feature_names=[f])
            for f in feats]
    ebc = EmbeddingBagCollection(tables=cfgs, device=torch.device("meta"))
    task = TwoTowerTrainTask(TwoTower(ebc, LAYERS, query_features=wl["query"], candidate_features=wl["cand"],
                                      device=device))
    _apply_optimizer_in_backward(RowWiseAdagrad, task.two_tower.ebc.parameters(), {"lr": LR})
    planner = EmbeddingShardingPlanner(topology=Topology(world_size=world, compute_device="cuda"),
                                       constraints={f"t_{f}": ParameterConstraints(sharding_types=[wl["sharding"][f]])
                                                    for f in feats})
    plan = planner.collective_plan(task, get_default_sharders(), dist.group.WORLD)
    model = DistributedModelParallel(module=task, device=device, plan=plan)
    sebc = model.module.two_tower.ebc
    assert isinstance(sebc, ShardedEmbeddingBagCollection)
    optimizer = KeyedOptimizerWrapper(dict(model.named_parameters()), lambda p: torch.optim.Adam(p, lr=0.01))
    pipeline = TrainPipelineSparseDist(model, optimizer, device)
    towers = [model.module.two_tower.query_proj, model.module.two_tower.candidate_proj]
    tower_params = [p for tw in towers for l in tw._mlp for p in (l._linear.weight, l._linear.bias)]

    allb = {(r, s): make_batch(wl, B, r, s) for r in range(world) for s in range(S)}
    touched = []
    for i, f in enumerate(feats):  # one table per feature
        touched.append(torch.unique(torch.cat([feature_ids(v, l, i, B) for (v, l, _) in allb.values()])))

    def snapshot():
        """rank 0: {table: (w [U, D], s [U])} of the touched rows, the flat tower params, Adam's
        moments (flat) and step; None elsewhere. Collective."""
        torch.cuda.synchronize()
        local = {}
        for (t, lo, n) in sebc._local_tables:
            u = touched[t]
            sel = (u >= lo) & (u < lo + n)
            if not bool(sel.any()):
                continue
            i = sebc._local_index[t]
            idx = (u[sel] - lo).to(device)
            local[t] = (sel, sebc._ts.table_view(i)[idx].cpu(), sebc._ts.state_view(i)[idx].cpu())
        got = [None] * world if rank == 0 else None
        dist.gather_object(local, got, dst=0)
        if rank != 0:
            return None
        tabs = {}
        for t in range(F):
            w = torch.full((touched[t].numel(), D), float("nan"))
            s_ = torch.full((touched[t].numel(),), float("nan"))
            for part in got:
                if t in part:
                    sel, pw, ps = part[t]
                    w[sel], s_[sel] = pw, ps
            assert not torch.isnan(w).any(), f"table {t}: touched rows missing from the shards"
            tabs[t] = (w, s_)
        flat = torch.cat([p.detach().reshape(-1).cpu() for p in tower_params])
        st = [optimizer.state.get(p, {}) for p in tower_params]
        if st[0]:
            m = torch.cat([x["exp_avg"].reshape(-1).cpu() for x in st])
            v = torch.cat([x["exp_avg_sq"].reshape(-1).cpu() for x in st])
        else:
            m, v = torch.zeros_like(flat), torch.zeros_like(flat)
        return tabs, flat, m, v

    def batches():
        for s in range(S):
            v, l, lab = allb[(rank, s)]
            yield Batch(dense_features=torch.zeros(1), sparse_features=KeyedJaggedTensor.from_lengths_sync(feats, v, l),
                        labels=lab)

    snaps = [snapshot()]
    outs = []
    it = batches()
    pipeline._model.train()
    for s in range(S):
        loss, logits, _ = pipeline.progress(it)
        outs.append((float(loss), logits.cpu()))
        snaps.append(snapshot())
        if rank == 0:
            print(f"trained step {s} (world {world})", flush=True)
    got_outs = [None] * world if rank == 0 else None
    dist.gather_object(outs, got_outs, dst=0)
    ok = True
    if rank == 0:
        ok = check(wl, B, S, world, feats, allb, touched, snaps, got_outs)
    flag = torch.tensor([1 if ok else 0])
    dist.broadcast(flag, src=0)
    del pipeline, model
    torch.cuda.synchronize()
    dist.destroy_process_group()
    if rank == 0:
        print("DMP-MULTIPROC-OK" if ok else "DMP-MULTIPROC-FAIL", flush=True)
    return 0 if int(flag) else 1


def check(wl, B, S, W, feats, allb, touched, snaps, got_outs):
    from tower_emul import acc_err, check_adagrad, check_adam, check_within, emulate_bounds, split_params

    F = len(feats)
    Fq = len(wl["query"])
    in_dims = [Fq * D, (F - Fq) * D]
    qi = [feats.index(f) for f in wl["query"]]
    ci = [feats.index(f) for f in wl["cand"]]
    for s in range(S):
        tabs, flat, m0, v0 = snaps[s]
        tabs1, flat1, m1, v1 = snaps[s + 1]
        prm = split_params(flat, in_dims, LAYERS)
        dx_rows = [[] for _ in range(F)]
        dx_eb = [[] for _ in range(F)]
        lk = [[] for _ in range(F)]
        gsum = [torch.zeros(p.numel(), dtype=torch.float64) for p in prm]
        esum = [torch.zeros(p.numel(), dtype=torch.float64) for p in prm]
        for r in range(W):
            v, lengths, lab = allb[(r, s)]
            pooled, eps_x, bag_of = [], [], []
            for i in range(F):
                ids = feature_ids(v, lengths, i, B)
                lens = lengths[i * B:(i + 1) * B].to(torch.int64)
                off = torch.zeros(B + 1, dtype=torch.int64)
                off[1:] = torch.cumsum(lens, 0)
                c = torch.searchsorted(touched[i], ids)
                w = tabs[i][0]
                pooled.append(torch.nn.functional.embedding_bag(c, w, off, mode="sum", include_last_offset=True))
                sq = torch.nn.functional.embedding_bag(c, w.double() ** 2, off, mode="sum", include_last_offset=True)
                e = acc_err(sq.sqrt(), pooled[-1].double(), int(max(1, int(lens.max()))))
                e[lens <= 1] = 0.0  # a single row is copied, not summed
                eps_x.append(e)
                bag = torch.repeat_interleave(torch.arange(B), lens)
                bag_of.append(bag)
                lk[i].append(c)
            xq = torch.cat([pooled[i] for i in qi], 1)
            xc = torch.cat([pooled[i] for i in ci], 1)
            exq = torch.cat([eps_x[i] for i in qi], 1)
            exc = torch.cat([eps_x[i] for i in ci], 1)
            (lg, e_lg), loss, dxs, gw, amb = emulate_bounds(xq, xc, prm, LAYERS, lab, ex=[exq, exc])
            got_loss, got_logits = got_outs[r][s]
            check_within(got_logits, lg, e_lg, f"step {s} rank {r} logits")
            okr = ~amb
            rel = ((got_logits.double() - lg).abs() / lg.abs().clamp_min(1e-30))[okr]
            assert float(rel.max()) <= 5e-3, f"step {s} rank {r}: logit relative error {float(rel.max()):.3g}"
            np.testing.assert_allclose(got_loss, float(loss), rtol=1e-4)
            for t, idx in ((0, qi), (1, ci)):
                for j, i in enumerate(idx):
                    cols = slice(j * D, (j + 1) * D)
                    dx_rows[i].append(dxs[t][0][:, cols][bag_of[i]])
                    dx_eb[i].append(dxs[t][1][:, cols][bag_of[i]])
            for j, (g, e) in enumerate(gw):
                gsum[j] += g.reshape(-1)
                esum[j] += e.reshape(-1)
            print(f"step {s} rank {r}: loss {got_loss:.6f}, logits max rel {float(rel.max()):.2e}, "
                  f"ambiguous rows {int(amb.sum())}", flush=True)
        # tables: RowWiseAdagrad on the SUM over ranks of the pooled gradients (TorchRec sharded EBC)
        for i in range(F):
            inv = torch.cat(lk[i])
            w_after, s_after = tabs1[i]
            check_adagrad(w_after, s_after, tabs[i][0], tabs[i][1], inv, torch.cat(dx_rows[i]), torch.cat(dx_eb[i]),
                          LR, 1e-10, f"step {s} table {feats[i]}")
        # towers: Adam on the MEAN over ranks (DDP), the fp32 all-reduce adds its own rounding
        g = torch.cat(gsum) / W
        e = torch.cat(esum) / W + 4 * W * 2.0 ** -24 * g.abs()
        check_adam(flat, m0, v0, s + 1, g, e, flat1, m1, v1, 0.01, what=f"step {s}")
        print(f"step {s}: tables and towers within the bounds", flush=True)
    return True


if __name__ == "__main__":
    from child_util import child_main

    child_main(main)
