"""World-size-2 CPU test of the reference's whole training / evaluation loop over the torchrec API
(03_model_training.py:770-840 main/train, :504-566 evaluate) through DistributedModelParallel on a
gloo process group: DMP shards the EmbeddingBagCollection (one table ROW_WISE, one TABLE_WISE, a
shared table), wraps the towers in DDP, and TrainPipelineSparseDist.progress trains 3 steps and then
evaluates in eval mode, each rank on its own batches. The local lookups use the test's oracle-backed
backend (tests/cpu_lookup_backend.py, injected through the sharder); the towers are plain torch
Linear + ReLU stacks (torchrec MLP semantics, ReLU on every layer) since the product's MLP is HIP-only.

The single-process reference it is checked against: per rank, the forward and the mean-BCE
gradient of that rank's batch (torch autograd on CPU, nn.EmbeddingBag sums); the towers step Adam on
the MEAN of the ranks' gradients (DDP), the tables take row-wise Adagrad on the SUM of the ranks'
gradients (TorchRec's sharded EBC: every rank's pooled gradient reaches the owner). Evaluation:
per-rank average loss = sum of batch losses / samples (the reference's quirk, 03:549-559) and the
AUROC of all ranks' predictions (torchmetrics' sync on compute)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

TABLES = [("t_user", 300, ["user_id"]), ("t_item", 500, ["product_id"]), ("t_shared", 40, ["u_tag", "i_tag"])]
QUERY = ["user_id", "u_tag"]
CAND = ["product_id", "i_tag"]
SHARDING = {"t_user": "row_wise", "t_item": "table_wise", "t_shared": "table_wise"}
D, B, LR, LAYERS, W = 8, 16, 0.05, [12, 6], 2
KEYS = [f for _, _, fs in TABLES for f in fs]
FTAB = [i for i, (_, _, fs) in enumerate(TABLES) for _ in fs]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tables0():
    g = torch.Generator().manual_seed(5)
    return [torch.empty(r, D).uniform_(-0.5, 0.5, generator=g) for _, r, _ in TABLES]


def _towers0():
    torch.manual_seed(9)
    mk = lambda i: nn.Sequential(*[m for a, b in zip([i] + LAYERS[:-1], LAYERS) for m in (nn.Linear(a, b), nn.ReLU())])  # noqa: E731
    return mk(D * len(QUERY)), mk(D * len(CAND))


def _batch(rank, step):
    """(values int64, lengths int32 [F * B], labels int32 [B]) of rank's step (steps 3, 4: eval)."""
    g = torch.Generator().manual_seed(1000 * rank + step)
    lengths = torch.randint(0, 4, (len(KEYS) * B,), generator=g).to(torch.int32)
    lengths[:3] = 0  # empty bags
    rows = [r for _, r, _ in TABLES]
    vals = [torch.randint(0, rows[FTAB[i // B]], (int(lengths[i]),), generator=g) for i in range(len(KEYS) * B)]
    return torch.cat(vals).to(torch.int64), lengths, torch.randint(0, 2, (B,), generator=g).to(torch.int32)


class _Tower(nn.Module):
    def __init__(self, seq):
        super().__init__()
        self._mlp = seq

    def forward(self, x):
        return self._mlp(x)


class _TwoTower(nn.Module):
    """03_model_training.py:395-437 with several features per tower (the ray-tune variant)."""

    def __init__(self, ebc, q, c):
        super().__init__()
        self.ebc = ebc
        self.query_proj = _Tower(q)
        self.candidate_proj = _Tower(c)

    def forward(self, kjt):
        kt = self.ebc(kjt)
        q = self.query_proj(torch.cat([kt[f] for f in QUERY], dim=1))
        c = self.candidate_proj(torch.cat([kt[f] for f in CAND], dim=1))
        return q, c


class _TrainTask(nn.Module):
    """03_model_training.py:440-455."""

    def __init__(self, two_tower):
        super().__init__()
        self.two_tower = two_tower
        self.loss_fn = nn.BCEWithLogitsLoss()

    def forward(self, batch):
        q, c = self.two_tower(batch.sparse_features)
        logits = (q * c).sum(dim=1).squeeze()
        loss = self.loss_fn(logits, batch.labels.float())
        return loss, (loss.detach(), logits.detach(), batch.labels.detach())


def _worker(rank, port, q):
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    dist.init_process_group("gloo", rank=rank, world_size=W, init_method=f"tcp://127.0.0.1:{port}")
    try:
        from torch.distributed.optim import _apply_optimizer_in_backward

        from cpu_lookup_backend import CpuLookupBackend
        from two_tower_recommender_model_amd.metrics import AUROC
        from two_tower_recommender_model_amd.torchrec.datasets.utils import Batch
        from two_tower_recommender_model_amd.torchrec.distributed.embeddingbag import (
            EmbeddingBagCollectionSharder, ShardedEmbeddingBagCollection)
        from two_tower_recommender_model_amd.torchrec.distributed.model_parallel import DistributedModelParallel
        from two_tower_recommender_model_amd.torchrec.distributed.planner import (EmbeddingShardingPlanner,
                                                                                   ParameterConstraints, Topology)
        from two_tower_recommender_model_amd.torchrec.distributed.train_pipeline import TrainPipelineSparseDist
        from two_tower_recommender_model_amd.torchrec.modules.embedding_configs import EmbeddingBagConfig
        from two_tower_recommender_model_amd.torchrec.modules.embedding_modules import EmbeddingBagCollection
        from two_tower_recommender_model_amd.torchrec.optim.keyed import KeyedOptimizerWrapper
        from two_tower_recommender_model_amd.torchrec.optim.rowwise_adagrad import RowWiseAdagrad
        from two_tower_recommender_model_amd.torchrec.sparse.jagged_tensor import KeyedJaggedTensor

        cpu = torch.device("cpu")
        cfgs = [EmbeddingBagConfig(name=n, embedding_dim=D, num_embeddings=r, feature_names=fs) for n, r, fs in TABLES]
        ebc = EmbeddingBagCollection(tables=cfgs, device=cpu)
        with torch.no_grad():
            for (n, _, _), w in zip(TABLES, _tables0()):
                ebc.embedding_bags[n].weight.copy_(w)
        task = _TrainTask(_TwoTower(ebc, *_towers0()))
        _apply_optimizer_in_backward(RowWiseAdagrad, task.two_tower.ebc.parameters(), {"lr": LR})
        sharders = [EmbeddingBagCollectionSharder(lookup_backend=CpuLookupBackend())]
        planner = EmbeddingShardingPlanner(topology=Topology(world_size=W, compute_device="cpu"),
                                           constraints={n: ParameterConstraints(sharding_types=[s])
                                                        for n, s in SHARDING.items()})
        plan = planner.collective_plan(task, sharders, dist.group.WORLD)
        model = DistributedModelParallel(module=task, device=cpu, plan=plan, sharders=sharders)
        assert isinstance(model.module.two_tower.ebc, ShardedEmbeddingBagCollection)
        optimizer = KeyedOptimizerWrapper(dict(model.named_parameters()), lambda p: torch.optim.Adam(p, lr=0.01))
        pipeline = TrainPipelineSparseDist(model, optimizer, cpu)

        def batches(steps):
            for s in steps:
                v, l, lab = _batch(rank, s)
                yield Batch(dense_features=torch.zeros(1),
                            sparse_features=KeyedJaggedTensor.from_lengths_sync(KEYS, v, l), labels=lab)

        out = {"train": []}
        it = batches(range(3))
        pipeline._model.train()
        while True:  # train() loop, 03:612-630
            try:
                loss, logits, _ = pipeline.progress(it)
            except StopIteration:
                break
            out["train"].append((float(loss), logits.numpy().copy()))
        # gather_and_get_state_dict (03:474-495, restated): ShardedTensors gathered to rank 0
        from torch.distributed._shard.sharded_tensor import ShardedTensor

        sd = {}
        for k, v in model.module.two_tower.state_dict().items():
            if isinstance(v, ShardedTensor):
                full = torch.zeros(v.size()) if rank == 0 else None
                v.gather(0, full)
                if rank == 0:
                    sd[k] = full.numpy().copy()
            elif rank == 0:
                sd[k] = v.detach().numpy().copy()
        out["sd"] = sd
        # evaluate() (03:504-566, restated)
        pipeline._model.eval()
        auroc = AUROC(task="binary").to(cpu)
        total_loss, total_samples = torch.tensor(0.0), 0
        it = batches([3, 4])
        with torch.no_grad():
            while True:
                try:
                    _loss, logits, labels = pipeline.progress(it)
                    auroc(torch.sigmoid(logits), labels)
                    total_loss += _loss.detach()
                    total_samples += len(labels)
                except StopIteration:
                    break
        out["eval"] = (float(total_loss / total_samples), float(auroc.compute()))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _reference():
    """The same 3 steps + evaluation in one process (see the module docstring)."""
    from oracle import ref
    from two_tower_recommender_model_amd.metrics import binary_auroc

    tables = [w.clone().requires_grad_(True) for w in _tables0()]
    states = [torch.zeros(r) for _, r, _ in TABLES]
    qt, ct = _towers0()
    dense = list(qt.parameters()) + list(ct.parameters())
    opt = torch.optim.Adam(dense, lr=0.01)

    def forward(rank, step):
        v, l, lab = _batch(rank, step)
        off = torch.from_numpy(ref.complete_cumsum(l.numpy())).to(torch.int64)
        cols = {}
        for f, name in enumerate(KEYS):
            o = off[f * B:(f + 1) * B + 1]
            cols[name] = nn.functional.embedding_bag(v[o[0]:o[-1]], tables[FTAB[f]], o[:-1] - o[0], mode="sum")
        q = qt(torch.cat([cols[f] for f in QUERY], 1))
        c = ct(torch.cat([cols[f] for f in CAND], 1))
        logits = (q * c).sum(1)
        return nn.functional.binary_cross_entropy_with_logits(logits, lab.float()), logits, lab

    want = {r: [] for r in range(W)}
    for s in range(3):
        gsum = [torch.zeros_like(t) for t in tables]
        dgrad = [torch.zeros_like(p) for p in dense]
        for r in range(W):
            loss, logits, _ = forward(r, s)
            grads = torch.autograd.grad(loss, tables + dense)
            want[r].append((float(loss.detach()), logits.detach().numpy().copy()))
            for i in range(len(tables)):
                gsum[i] += grads[i]
            for i, gd in enumerate(grads[len(tables):]):
                dgrad[i] += gd
        with torch.no_grad():
            for t, st, gr in zip(tables, states, gsum):
                ref.rowwise_adagrad(t, st, gr, LR, 1e-10)
        opt.zero_grad()
        for p, gd in zip(dense, dgrad):
            p.grad = gd / W  # DDP: mean over ranks
        opt.step()
    ev = {}
    preds, labels = [], []
    with torch.no_grad():
        for r in range(W):
            tot, n = 0.0, 0
            for s in (3, 4):
                loss, logits, lab = forward(r, s)
                tot += float(loss)
                n += B
                preds.append(torch.sigmoid(logits))
                labels.append(lab)
            ev[r] = tot / n
    auc = float(binary_auroc(torch.cat(preds), torch.cat(labels)))
    return want, [t.detach() for t in tables], (qt, ct), ev, auc


def test_dmp_train_eval_world2_vs_reference():
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(W)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(W))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want, tables, (qt, ct), ev, auc = _reference()
    for r in range(W):
        assert len(got[r]["train"]) == 3
        for (gl, glog), (wl, wlog) in zip(got[r]["train"], want[r]):
            assert gl == pytest.approx(wl, rel=1e-5)
            np.testing.assert_allclose(glog, wlog, rtol=1e-5, atol=1e-6)
    sd = got[0]["sd"]
    for (n, _, _), t in zip(TABLES, tables):
        np.testing.assert_allclose(sd[f"ebc.embedding_bags.{n}.weight"], t.numpy(), rtol=1e-5, atol=1e-6)
    for name, mod in (("query_proj", qt), ("candidate_proj", ct)):
        for k, v in mod.state_dict().items():
            np.testing.assert_allclose(sd[f"{name}._mlp.{k}"], v.numpy(), rtol=1e-5, atol=1e-6)
    for r in range(W):
        assert got[r]["eval"][0] == pytest.approx(ev[r], rel=1e-5)  # per-rank average loss
        assert got[r]["eval"][1] == pytest.approx(auc, abs=1e-6)   # AUROC over every rank's predictions
