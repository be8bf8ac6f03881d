"""The reference's own training loop on the fused kernels: ``TrainPipelineSparseDist.progress``
(03_model_training.py:618, :648) dispatched to the production ring of ``FusedTwoTowerStep``.

The loop the reference runs is ``DistributedModelParallel`` -> EBC lookup -> ``MLP`` Perceptrons ->
autograd -> RowWiseAdagrad in backward -> ``KeyedOptimizerWrapper(Adam)`` (03:612-625, :791-829).
Through the torchrec shim that is a sequence of per-op launches (pooled forward, per-layer GEMMs,
dot + BCE, their backwards, the dedup + Adagrad kernels, torch's Adam). When the model is the
reference's two-tower shape, every step of that sequence is what one fused ring step computes, so
the pipeline hands the batches to ``FusedTwoTowerStep`` instead:

* the step ADOPTS the model's storage: the tables and their row-wise Adagrad state are the
  EmbeddingBagCollection's (or the one-rank ShardedEmbeddingBagCollection's) TableSet, the tower
  parameters become views of the step's flat parameter buffer (``Parameter.data`` re-pointed, so
  ``state_dict()``, eval-mode forwards and checkpoints see every update), and the Adam moments of
  the wrapped ``torch.optim.Adam`` become views of the step's moment buffers;
* each batch's single-hot KJT (transform_to_torchrec_batch's output, 03:353-380) is turned into the
  step's id columns on the device (``tt_kjt_single_hot_cols``; id 0 dropped = empty bag) in one of
  ``depth`` resident slots; slot k's HIP graph is one ring step on slot k that files slot k+1's
  dedup table (the ring needs the next batch, which the pipeline has already fetched);
* progress() returns ``(loss, logits, labels)`` device tensors, as the reference's task does.

Conditions (else the generic per-op path runs, unchanged): world size 1 (the fused sharded step is a
separate API), ``TwoTowerTrainTask(TwoTower)`` with one feature per tower, equal embedding dims of
64 or 128, towers [128, 64] in bf16 (the production precision; the fp32 parity mode stays generic),
fused RowWiseAdagrad on the tables, Adam with default betas / eps and no weight decay, SUM pooling,
a KJT whose keys are (query feature, candidate feature) with bags of at most one id and a batch size
that is a multiple of 8. A batch that does not fit (e.g. a smaller last batch of an epoch) runs
through the generic path between fused steps, with the Adam step count synchronised both ways.
``TT_DROPIN_FUSED=0`` turns the dispatch off.
"""
from __future__ import annotations

import os
from typing import Any, Iterator, List, Optional, Tuple

import torch
from torch import nn

from . import _lib, ops


def _named(obj, cls_name: str) -> bool:
    return type(obj).__name__ == cls_name


class _Item:
    __slots__ = ("batch", "slot", "parity", "labels", "primed")

    def __init__(self, batch, slot=None, parity=0, labels=None):
        self.batch = batch
        self.slot = slot
        self.parity = parity
        self.labels = labels
        self.primed = False


class FusedDropin:
    """Built by ``TrainPipelineBase`` at its first training ``progress``; ``None`` (with a reason)
    when the model / optimizer is not the shape the fused ring runs."""

    def __init__(self, pipeline, task, ebc, ts, fused_cfg, towers: Tuple[nn.Module, nn.Module], adam,
                 feats: List[str], dims: List[int], depth: int = 16, fresh_outputs: bool = False):
        self.pipeline = pipeline
        self.task = task
        self.ebc = ebc
        self.ts = ts
        self.fused_cfg = fused_cfg
        self.towers = towers
        self.adam = adam
        self.feats = feats
        self.dims = dims
        self.depth = int(depth)
        self.fresh_outputs = bool(fresh_outputs)
        self.device = pipeline._device
        self.step = None  # FusedTwoTowerStep, built at the first fusable batch (its B)
        self.cur: Optional[_Item] = None
        self.nxt: Optional[_Item] = None
        self.k = 0  # fused batches staged so far (slot = k % depth, ring parity = k % 2)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.steps_fused = 0
        self.steps_generic = 0

    # ---- applicability ------------------------------------------------------------------------
    @classmethod
    def build(cls, pipeline) -> Tuple[Optional["FusedDropin"], str]:
        if os.environ.get("TT_DROPIN_FUSED", "1") == "0":
            return None, "TT_DROPIN_FUSED=0"
        if pipeline._device.type != "cuda":
            return None, "not a GPU pipeline"
        import torch.distributed as dist

        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        model = pipeline._model
        task = getattr(model, "module", model)
        if world == 1 and getattr(model, "_ddp", None) is not None:
            return None, "DDP-wrapped dense modules"
        if not _named(task, "TwoTowerTrainTask") or not hasattr(task, "two_tower"):
            return None, "the model is not a TwoTowerTrainTask"
        loss_fn = getattr(task, "loss_fn", None)
        if loss_fn is not None and not (isinstance(loss_fn, nn.BCEWithLogitsLoss) and loss_fn.reduction == "mean"
                                        and loss_fn.weight is None and loss_fn.pos_weight is None):
            return None, "the task's loss is not BCEWithLogitsLoss(mean)"
        tt = task.two_tower
        if not _named(tt, "TwoTower"):
            return None, "the task's tower module is not a TwoTower"
        qf, cf = list(getattr(tt, "_feature_names_query", [])), list(getattr(tt, "_candidate_feature_names", []))
        if len(qf) != 1 or len(cf) != 1:
            return None, "one feature per tower only"
        ebc = tt.ebc
        from .torchrec.distributed.embeddingbag import ShardedEmbeddingBagCollection
        from .torchrec.modules.embedding_modules import EmbeddingBagCollection

        feats = [qf[0], cf[0]]
        sharded = None  # world > 1: (sharding, owner) per feature
        if world > 1:
            if not isinstance(ebc, ShardedEmbeddingBagCollection) or ebc._W != world:
                return None, "world size > 1 without a ShardedEmbeddingBagCollection over every rank"
            if ebc._be is not ops.HIP_BACKEND:
                return None, "the sharded EBC does not run on the HIP lookup backend"
            if ebc._pooling != _lib.TT_POOL_SUM or ebc._feature_names != feats or ebc._f_table != [0, 1]:
                return None, "EBC features are not (query, candidate) with SUM pooling, one table each"
            sharded = []
            for f in range(2):
                if f in ebc._rw_feats:
                    sharded.append(("row_wise", 0))
                else:
                    sharded.append(("table_wise", next(o for o in range(world) if f in ebc._tw_by_owner[o])))
            cfg = ebc._fused
            dims = list(ebc._dims)
            ts = ebc._ts
        elif isinstance(ebc, ShardedEmbeddingBagCollection):
            if ebc._W != 1 or ebc._ts is None:
                return None, "sharded over more than one rank"
            if ebc._pooling != _lib.TT_POOL_SUM or ebc._feature_names != feats:
                return None, "EBC features are not (query, candidate) with SUM pooling"
            tabs = [ebc._local_index.get(ebc._f_table[f]) for f in range(2)]
            if tabs != [0, 1] or ebc._ts.T != 2:
                return None, "EBC tables are not one per tower"
            ts, cfg = ebc._ts, ebc._fused
        elif isinstance(ebc, EmbeddingBagCollection):
            if ebc._pooling != _lib.TT_POOL_SUM or ebc._feature_names != feats or ebc._feature_table != [0, 1]:
                return None, "EBC features are not (query, candidate) with SUM pooling"
            if not ebc._bound_to_ts() or ebc._ts.device != pipeline._device:
                ebc._materialize(pipeline._device)
            ts, cfg = ebc._ts, ebc._fused_cfg()
        else:
            return None, "the tower module's ebc is not an EmbeddingBagCollection"
        if cfg is None:
            return None, "tables without the fused in-backward RowWiseAdagrad"
        if sharded is None:
            dims = [ts.dims[0], ts.dims[1]]
        if dims[0] != dims[1] or dims[0] not in (64, 128):
            return None, "embedding dims must be equal, 64 or 128"
        towers = (tt.query_proj, tt.candidate_proj)
        for mlp, d in zip(towers, dims):
            layers = list(getattr(mlp, "_mlp", []))
            if len(layers) != 2:
                return None, "towers must be MLP(layer_sizes=[128, 64])"
            shapes = [tuple(p._linear.weight.shape) for p in layers]
            if shapes != [(128, d), (64, 128)] or any(p._linear.bias is None for p in layers):
                return None, "towers must be MLP(layer_sizes=[128, 64]) with biases"
            if any(getattr(p, "precision", "bf16") != "bf16" for p in layers):
                return None, "fp32 tower precision (parity mode) runs the generic path"
        opt = pipeline._optimizer
        adam = getattr(opt, "_optimizer", opt)
        if not isinstance(adam, torch.optim.Adam):
            return None, "the optimizer is not (a wrapper of) torch.optim.Adam"
        for g in adam.param_groups:
            if (tuple(g["betas"]) != (0.9, 0.999) or g["eps"] != 1e-8 or g["weight_decay"] != 0 or g["amsgrad"]
                    or g.get("maximize", False)):
                return None, "Adam hyper-parameters other than the defaults"
        mlp_params = [p for m in towers for l in m._mlp for p in (l._linear.weight, l._linear.bias)]
        ids = {id(p) for p in mlp_params}
        table_ids = {id(p) for p in ebc.parameters()}  # updated in backward (grad None), or zero-size
        lrs = set()
        for g in adam.param_groups:
            for p in g["params"]:
                if id(p) in ids:
                    lrs.add(g["lr"])
                elif p.numel() and id(p) not in table_ids:
                    return None, "Adam holds parameters besides the towers and the fused tables"
        if len(lrs) != 1:
            return None, "the towers' Adam parameters do not share one learning rate"
        if sharded is not None:
            return FusedShardedDropin(pipeline, task, ebc, ts, cfg, towers, adam, feats, dims, sharded), \
                "fused sharded"
        return cls(pipeline, task, ebc, ts, cfg, towers, adam, feats, dims), "fused"

    def _adam_group(self) -> dict:
        w = self.towers[0]._mlp[0]._linear.weight
        for g in self.adam.param_groups:
            if any(p is w for p in g["params"]):
                return g
        raise _lib.TTError("dropin: tower parameters left the optimizer")

    def _adam_lr(self) -> float:
        return float(self._adam_group()["lr"])

    def fusable(self, batch) -> bool:
        kjt = getattr(batch, "sparse_features", None)
        if kjt is None or list(kjt.keys()) != self.feats:
            return False
        B = kjt.stride()
        if B < 8 or B % 8 or (self.step is not None and B != self.step.B):
            return False
        v = kjt.values()
        if v.numel() > 2 * B:  # a bag with more than one id somewhere: multi-hot
            return False
        if v.numel() and v.dtype not in (torch.int32, torch.int64):
            return False
        if self.step is not None and v.numel() and v.dtype != self.step.id_dtype:
            return False
        lab = batch.labels
        return (lab.numel() == B and lab.dtype in (torch.int32, torch.int64) and lab.is_contiguous()
                and lab.device == self.device and kjt.device() == self.device)

    # ---- the fused step, adopting the model's storage --------------------------------------------
    def _make_step(self, B: int, id_dtype: torch.dtype) -> None:
        from .fused import FusedTwoTowerStep

        ts, dev = self.ts, self.device
        lr_dense = self._adam_lr()
        st = FusedTwoTowerStep([ts.rows[0], ts.rows[1]], self.dims, [0], [1], [128, 64], B, dev,
                               lr_emb=self.fused_cfg["lr"], lr_dense=lr_dense, eps=self.fused_cfg["eps"],
                               id_dtype=id_dtype, tables=ts)
        if not st.ring_supported():
            raise _lib.TTError("dropin: the fused ring does not support this shape")
        # the towers' parameters -> views of the step's flat buffer (values copied first); Adam's
        # moments likewise (the flat layout is [W0, b0, W1, b1] of the query tower, then the
        # candidate tower's: FusedTwoTowerStep.qW / qb / cW / cb)
        views = [st.qW[0], st.qb[0], st.qW[1], st.qb[1], st.cW[0], st.cb[0], st.cW[1], st.cb[1]]
        params = [p for m in self.towers for l in m._mlp for p in (l._linear.weight, l._linear.bias)]
        o = 0
        steps = set()
        with torch.no_grad():
            for p, v in zip(params, views):
                v.copy_(p.detach())
                n = v.numel()
                s = self.adam.state.get(p)
                if s and "exp_avg" in s:
                    st.exp_avg[o:o + n].view_as(v).copy_(s["exp_avg"])
                    st.exp_avg_sq[o:o + n].view_as(v).copy_(s["exp_avg_sq"])
                    steps.add(int(float(s["step"])))
                o += n
        if len(steps) > 1:
            raise _lib.TTError("dropin: the towers' Adam step counts differ")
        n_adam = steps.pop() if steps else 0
        st.adam_state[0] = n_adam
        o = 0
        for p, v in zip(params, views):
            n = v.numel()
            p.data = v
            self.adam.state[p] = {"step": torch.tensor(float(n_adam)), "exp_avg": st.exp_avg[o:o + n].view_as(v),
                                  "exp_avg_sq": st.exp_avg_sq[o:o + n].view_as(v)}
            o += n
        st.sync_weights()
        self._params = params
        self.step = st
        D = self.depth
        idt = id_dtype
        self.slot_cols = [[torch.zeros(B, dtype=idt, device=dev) for _ in range(2)] for _ in range(D)]
        self.slot_labels = [torch.zeros(B, dtype=torch.int32, device=dev) for _ in range(D)]
        self.slot_logits = [torch.zeros(B, dtype=torch.float32, device=dev) for _ in range(D)]
        self.slot_loss = [torch.zeros((), dtype=torch.float32, device=dev) for _ in range(D)]
        self.zero_cols = [torch.zeros(B, dtype=idt, device=dev) for _ in range(2)]
        # the per-batch conversion's ctypes arguments, built once
        import ctypes as C

        self._lib = _lib.load()
        self._ne = (C.c_int64 * 2)(*st.num_embeddings)
        self._slot_ptrs = [_lib.ptr_array(c) for c in self.slot_cols]
        self._idt = _lib.id_dtype_code(idt)
        self._group = self._adam_group()
        self._capture()

    def _ring_step(self, slot: int, parity: int, next_cols) -> None:
        st = self.step
        keep = st.logits, st.loss
        st.logits, st.loss = self.slot_logits[slot], self.slot_loss[slot]
        try:
            st.ring_step(self.slot_cols[slot], self.slot_labels[slot], parity, next_cols)
        finally:
            st.logits, st.loss = keep

    def _capture(self) -> None:
        """Slot k's graph: the ring step on slot k (parity k % 2) filing slot k+1's dedup table."""
        st, D, dev = self.step, self.depth, self.device
        st._ring_ws()
        self.lr_captured = st.lr_dense
        self.graphs = []
        torch.cuda.synchronize(dev)
        for k in range(D):
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    self._ring_step(k, k % 2, self.slot_cols[(k + 1) % D])
            torch.cuda.current_stream(dev).wait_stream(s)
            _lib.graph_upload(g, dev)
            self.graphs.append(g)
        torch.cuda.synchronize(dev)

    # ---- staging -----------------------------------------------------------------------------
    def _fetch(self, it: Iterator) -> Optional[_Item]:
        try:
            batch = next(it)
        except StopIteration:
            return None
        batch = batch.to(self.device, non_blocking=True)
        if not self.fusable(batch):
            return _Item(batch)
        kjt = batch.sparse_features
        v = kjt.values()
        if self.step is None:
            # the first fusable batch fixes B and the id dtype; one synchronising check that its
            # bags are single-hot (later batches: the conversion's sticky error word)
            if int(kjt.lengths().max()) > 1 if kjt.lengths().numel() else False:
                return _Item(batch)
            self._make_step(kjt.stride(), v.dtype if v.numel() else torch.int64)
        k = self.k
        self.k += 1
        slot = k % self.depth
        offs = kjt.offsets()
        if offs.dtype != torch.int32:
            offs = offs.to(torch.int32)
        lab = batch.labels
        # ids -> slot columns and labels -> slot labels in one launch (shapes / dtypes checked by
        # fusable(); an empty values tensor is never read)
        _lib.check(self._lib.tt_kjt_single_hot_cols(
            2, self.step.B, v.data_ptr() if v.numel() else self.slot_cols[slot][0].data_ptr(), self._idt,
            offs.data_ptr(), self._ne, self._slot_ptrs[slot], self.err.data_ptr(), lab.data_ptr(),
            _lib.TT_I64 if lab.dtype == torch.int64 else _lib.TT_I32, self.slot_labels[slot].data_ptr(),
            torch.cuda.current_stream(self.device).cuda_stream), "kjt_single_hot_cols")
        return _Item(batch, slot, k % 2, lab)

    def check_errors(self) -> None:
        """Raise if any converted batch had a multi-id bag or an id out of range (one sync)."""
        e = int(self.err.item())
        if e:
            self.err.zero_()
            raise _lib.TTError(f"dropin: a KJT batch had {'a bag of several ids' if e & 1 else ''}"
                               f"{' and ' if e == 3 else ''}{'an id outside [0, N)' if e & 2 else ''} "
                               "(TorchRec's EBC takes ids in range; single-hot bags only on this path). The "
                               "fused ring trained on the converted batch (such a bag as an empty one) and on "
                               "every batch after it in this chunk: the tables, towers and optimizer state are "
                               "not what the reference's loop would hold — restore a checkpoint, or run such "
                               "data with TT_DROPIN_FUSED=0")

    def sync_optimizer_state(self) -> None:
        """torch Adam's per-parameter step count <- the fused step's (the moments are shared views);
        run at every chunk's end (StopIteration), so optimizer.state_dict() there is current."""
        if self.step is None:
            return
        n = torch.tensor(float(int(self.step.adam_state[0].item())))
        for q in self._params:
            self.adam.state[q]["step"] = n.clone()

    def pending(self) -> bool:
        return self.cur is not None

    def drain_to(self, pipeline) -> None:
        """Mode switch with batches staged (an eval progress mid-chunk): hand them back to the generic
        pipeline, unfiled (both dedup tables emptied)."""
        from .torchrec.distributed.train_pipeline import _Staged

        items = [x for x in (self.cur, self.nxt) if x is not None]
        self.cur = self.nxt = None
        if self.step is not None:
            self.step.ring_reset()
        if items:
            pipeline._cur = _Staged(items[0].batch, None)
            pipeline._next = _Staged(items[1].batch, None) if len(items) > 1 else None

    # ---- one progress() ----------------------------------------------------------------------
    def progress(self, it: Iterator) -> Any:
        if self.cur is None:
            self.cur = self._fetch(it)
            if self.cur is None:
                self.check_errors()
                self.sync_optimizer_state()
                raise StopIteration
            self.nxt = self._fetch(it)
        cur, nxt = self.cur, self.nxt
        if cur.slot is None:
            out = self._generic(cur.batch)
        else:
            out = self._fused(cur, nxt)
        self.cur, self.nxt = nxt, None
        if self.cur is not None:
            self.nxt = self._fetch(it)
        return out

    def _fused(self, cur: _Item, nxt: Optional[_Item]) -> Any:
        st = self.step
        lr = self._group["lr"]
        if lr != self.lr_captured:  # the plan carries Adam's lr: re-capture after a change
            st.lr_dense = float(lr)
            self._capture()
        if not cur.primed:
            st.ring_prime(self.slot_cols[cur.slot], cur.parity)
        if nxt is not None and nxt.slot is not None:
            self.graphs[cur.slot].replay()
            nxt.primed = True
        else:  # the next batch is not fused (or there is none yet): file nothing
            self._ring_step(cur.slot, cur.parity, self.zero_cols)
        self.steps_fused += 1
        loss, logits = self.slot_loss[cur.slot], self.slot_logits[cur.slot]
        if self.fresh_outputs:
            loss, logits = loss.clone(), logits.clone()
        return loss, logits, cur.labels

    def _generic(self, batch) -> Any:
        """A batch the fused step does not take: the per-op path, on the shared storage, with the Adam
        step count carried across (the moments are shared views)."""
        p = self.pipeline
        st = self.step
        if st is not None:
            n = int(st.adam_state[0].item())
            for q in self._params:
                self.adam.state[q]["step"] = torch.tensor(float(n))
        p._optimizer.zero_grad(set_to_none=True)
        losses, output = p._model(batch)
        torch.sum(losses, dim=0).backward()
        p._optimizer.step()
        if st is not None:
            st.adam_state[0] = n + 1
            st.sync_weights()  # the towers' bf16 copies of the updated fp32 parameters
        self.steps_generic += 1
        return output


class FusedShardedDropin:
    """The reference's loop at world size W > 1 (DistributedModelParallel over W processes, one GPU
    each, 03_model_training.py:812-815, :918) on the pipelined fused sharded step
    (``sharded.FusedShardedTwoTowerStep``): TrainPipelineSparseDist.progress hands each single-hot
    batch to the step, which trains the ShardedEmbeddingBagCollection's OWN shards (table-wise or
    row-wise per the DMP plan; ``ops.TableSet.view_of``) and the towers' parameters and Adam moments
    as views of its flat buffers (the DDP replicas: the step's fixed-order mean of the W tower
    gradients is DDP's all-reduce mean). Per step two fixed-size all-to-alls instead of the eager
    input_dist / output_dist / DDP collectives with their host-synchronised split sizes.

    The step is pipelined two batches deep (batch i+1's rows are gathered during step i, batch
    i+2's ids routed), so progress() looks two batches ahead; slot k's HIP graph (RCCL inside) is
    the step on slot k routing slot k+2. Every rank must take the same path for the same batch (the
    step is collective): the choice uses host metadata only (stride, value count, dtype), which the
    reference's loaders give every rank alike. A batch the step does not take (another batch size,
    multi-hot values) runs the generic DMP path between fused steps; the staged pipeline is dropped
    first. Segment capacities come from the first batch's routes (max over ranks x 1.5, at least
    1.5 B / W + 64); a later batch beyond them drops the excess lookups and sets a sticky flag
    that is checked (collectively) at every StopIteration, as is a bag of several ids."""

    def __init__(self, pipeline, task, ebc, ts, fused_cfg, towers, adam, feats, dims, sharded, depth: int = 8):
        import torch.distributed as dist

        self.pipeline = pipeline
        self.task = task
        self.ebc = ebc
        self.ts = ts
        self.fused_cfg = fused_cfg
        self.towers = towers
        self.adam = adam
        self.feats = feats
        self.dims = dims
        self.sharding = [s for s, _ in sharded]
        self.owners = [o for _, o in sharded]
        self.depth = int(depth)  # even: parity = slot % 2
        self.device = pipeline._device
        self.W = dist.get_world_size(ebc._pg)
        self.step = None
        self.queue: List[_Item] = []  # fetched batches: cur, nxt, nxt2
        self.k = 0
        self.staged = False  # the step holds batch queue[0]'s rows and the next batch's route
        self.dirty = False   # a fused step ran since the last reset (its dedup tables hold keys)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.steps_fused = 0
        self.steps_generic = 0
        self.graphs: List = []
        self.graph_mode = None

    # reuse of the single-GPU drop-in's helpers
    _adam_group = FusedDropin._adam_group
    _adam_lr = FusedDropin._adam_lr

    def fusable(self, batch) -> bool:
        kjt = getattr(batch, "sparse_features", None)
        if kjt is None or list(kjt.keys()) != self.feats:
            return False
        B = kjt.stride()
        if B < 8 or B % 8 or (self.step is not None and B != self.step.B):
            return False
        v = kjt.values()
        if v.numel() > 2 * B or (v.numel() and v.dtype not in (torch.int32, torch.int64)):
            return False
        if self.step is not None and v.numel() and v.dtype != self.step.id_dtype:
            return False
        lab = batch.labels
        return (lab.numel() == B and lab.dtype in (torch.int32, torch.int64) and lab.is_contiguous()
                and lab.device == self.device and kjt.device() == self.device)

    # ---- the step on the sharded EBC's storage ---------------------------------------------------
    def _make_step(self, batch) -> None:
        import ctypes as C

        import torch.distributed as dist

        from .sharded import FusedShardedTwoTowerStep, TorchComm, default_capacity

        kjt = batch.sparse_features
        B = kjt.stride()
        v = kjt.values()
        idt = v.dtype if v.numel() else torch.int64
        dev, W, ebc = self.device, self.W, self.ebc
        # every rank's first batch agrees on B and the id dtype (else: the generic path everywhere)
        agree = torch.tensor([B, -B, 1 if idt == torch.int64 else 0, -(1 if idt == torch.int64 else 0)],
                             dtype=torch.int64, device=dev)
        dist.all_reduce(agree, op=dist.ReduceOp.MAX, group=ebc._pg)
        if int(agree[0]) != -int(agree[1]) or int(agree[2]) != -int(agree[3]):
            raise _lib.TTError("dropin (sharded): the ranks' first batches differ in batch size or id dtype")
        N = [c.num_embeddings for c in ebc._embedding_bag_configs]
        D = self.dims[0]
        cols = self._cols_of(kjt, B)
        blocks = [-(-n // W) if s == "row_wise" else 0 for n, s in zip(N, self.sharding)]
        seg_owner = [o if s == "table_wise" else 0 for o, s in zip(self.owners, self.sharding)]
        from .sharded import segment_counts

        need = segment_counts(cols, N, blocks, seg_owner, W).max().reshape(1).to(dev)
        dist.all_reduce(need, op=dist.ReduceOp.MAX, group=ebc._pg)
        cap = max(default_capacity(B, W, factor=1.5), -(-int(need) * 3 // 2))
        cap = min(B, -(-cap // 8) * 8)
        local = [ebc._local_index.get(ebc._f_table[f]) for f in range(2)]
        tables = ops.TableSet.view_of(self.ts, local, [D, D], dev)
        comm = TorchComm(group=ebc._pg, always_collective=True)
        st = FusedShardedTwoTowerStep(comm, N, D, [128, 64], B, dev, sharding=self.sharding, tw_owners=self.owners,
                                      lr_emb=self.fused_cfg["lr"], lr_dense=self._adam_lr(),
                                      eps=self.fused_cfg["eps"], id_dtype=idt, capacity=cap, tables=tables)
        # the towers' parameters -> views of the step's flat buffer; Adam's moments likewise
        views = [x for layers in st.layer_views() for wb in layers for x in wb]
        params = [p for m in self.towers for l in m._mlp for p in (l._linear.weight, l._linear.bias)]
        steps, o = set(), 0
        with torch.no_grad():
            for p, vw in zip(params, views):
                vw.copy_(p.detach())
                n = vw.numel()
                s = self.adam.state.get(p)
                if s and "exp_avg" in s:
                    st.exp_avg[o:o + n].view_as(vw).copy_(s["exp_avg"])
                    st.exp_avg_sq[o:o + n].view_as(vw).copy_(s["exp_avg_sq"])
                    steps.add(int(float(s["step"])))
                o += n
        if len(steps) > 1:
            raise _lib.TTError("dropin: the towers' Adam step counts differ")
        n_adam = steps.pop() if steps else 0
        st.adam_state[0] = n_adam
        o = 0
        for p, vw in zip(params, views):
            n = vw.numel()
            p.data = vw
            self.adam.state[p] = {"step": torch.tensor(float(n_adam)), "exp_avg": st.exp_avg[o:o + n].view_as(vw),
                                  "exp_avg_sq": st.exp_avg_sq[o:o + n].view_as(vw)}
            o += n
        st.towers.update(st.params, do_adam=False)
        self._params = params
        self.step = st
        Dp = self.depth
        self.slot_cols = [[torch.zeros(B, dtype=idt, device=dev) for _ in range(2)] for _ in range(Dp)]
        self.slot_labels = [torch.zeros(B, dtype=torch.int32, device=dev) for _ in range(Dp)]
        self.slot_logits = [torch.zeros(B, dtype=torch.float32, device=dev) for _ in range(Dp)]
        self.slot_loss = [torch.zeros((), dtype=torch.float32, device=dev) for _ in range(Dp)]
        self.zero_cols = [torch.zeros(B, dtype=idt, device=dev) for _ in range(2)]
        self._lib = _lib.load()
        self._ne = (C.c_int64 * 2)(*N)
        self._slot_ptrs = [_lib.ptr_array(c) for c in self.slot_cols]
        self._idt = _lib.id_dtype_code(idt)
        self._group = self._adam_group()
        # graphs with the collectives inside need RCCL (gloo collectives are not capturable)
        self.graph_mode = dist.get_backend(ebc._pg) == "nccl"
        if self.graph_mode:
            try:
                self._capture()
            except Exception as e:  # noqa: BLE001 - the same collectives run eagerly
                import sys

                print(f"dropin (sharded): graph capture with collectives refused ({e}); eager steps", file=sys.stderr)
                torch.cuda.synchronize(dev)
                self.graphs, self.graph_mode = [], False

    def _cols_of(self, kjt, B):
        """Host-side view of a batch's single-hot ids as id columns (the capacity probe only)."""
        o = kjt.offsets().to(torch.int64)
        v = kjt.values()
        cols = []
        for f in range(2):
            ln = o[f * B + 1:(f + 1) * B + 1] - o[f * B:(f + 1) * B]
            c = torch.zeros(B, dtype=torch.int64, device=v.device)
            idx = o[f * B:(f + 1) * B][ln > 0]
            c[ln > 0] = v[idx].to(torch.int64) % self.ebc._embedding_bag_configs[f].num_embeddings
            c[(ln > 0) & (c == 0)] = self.ebc._embedding_bag_configs[f].num_embeddings  # row 0 kept
            cols.append(c)
        return cols

    def _pipelined(self, slot: int, parity: int, next2) -> None:
        st = self.step
        keep = st.logits, st.loss
        st.logits, st.loss = self.slot_logits[slot], self.slot_loss[slot]
        try:
            st.step_pipelined(self.slot_labels[slot], parity, next2)
        finally:
            st.logits, st.loss = keep

    def _capture(self) -> None:
        """Slot k's graph: the pipelined step on slot k (parity k % 2) routing slot k + 2."""
        st, Dp, dev = self.step, self.depth, self.device
        self.lr_captured = st.lr_dense
        st.comm.retire()
        self.graphs = []
        torch.cuda.synchronize(dev)
        for k in range(Dp):
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    self._pipelined(k, k % 2, self.slot_cols[(k + 2) % Dp])
            torch.cuda.current_stream(dev).wait_stream(s)
            _lib.graph_upload(g, dev)
            self.graphs.append(g)
        torch.cuda.synchronize(dev)

    # ---- staging -----------------------------------------------------------------------------
    def _fetch(self, it: Iterator) -> Optional[_Item]:
        try:
            batch = next(it)
        except StopIteration:
            return None
        batch = batch.to(self.device, non_blocking=True)
        if not self.fusable(batch):
            return _Item(batch)
        kjt = batch.sparse_features
        if self.step is None:
            if int(kjt.lengths().max()) > 1 if kjt.lengths().numel() else False:
                return _Item(batch)
            self._make_step(batch)
        v = kjt.values()
        k = self.k
        self.k += 1
        slot = k % self.depth
        offs = kjt.offsets()
        if offs.dtype != torch.int32:
            offs = offs.to(torch.int32)
        lab = batch.labels
        _lib.check(self._lib.tt_kjt_single_hot_cols(
            2, self.step.B, v.data_ptr() if v.numel() else self.slot_cols[slot][0].data_ptr(), self._idt,
            offs.data_ptr(), self._ne, self._slot_ptrs[slot], self.err.data_ptr(), lab.data_ptr(),
            _lib.TT_I64 if lab.dtype == torch.int64 else _lib.TT_I32, self.slot_labels[slot].data_ptr(),
            torch.cuda.current_stream(self.device).cuda_stream), "kjt_single_hot_cols")
        return _Item(batch, slot, k % 2, lab)

    def _fill(self, it: Iterator) -> None:
        while len(self.queue) < 3:
            x = self._fetch(it)
            if x is None:
                break
            self.queue.append(x)

    def _reset(self) -> None:
        if self.step is not None and self.dirty:
            self.step.reset_pipeline()
        self.staged = self.dirty = False

    def check_errors(self) -> None:
        """Raise (on every rank) if a converted batch had a multi-id bag or an id out of range, or a
        route overflowed a segment's capacity (collective)."""
        import torch.distributed as dist

        e = self.err.clone()
        dist.all_reduce(e, op=dist.ReduceOp.MAX, group=self.ebc._pg)
        if self.step is not None:
            self.step.check()
        if int(e.item()):
            self.err.zero_()
            raise _lib.TTError("dropin (sharded): a KJT batch had a bag of several ids or an id outside [0, N) "
                               "(single-hot bags only on this path). The fused step trained on the converted "
                               "batch and the ones after it in this chunk: the model state is not what the "
                               "reference's loop would hold — restore a checkpoint, or run such data with "
                               "TT_DROPIN_FUSED=0")

    def sync_optimizer_state(self) -> None:
        if self.step is None:
            return
        n = torch.tensor(float(int(self.step.adam_state[0].item())))
        for q in self._params:
            self.adam.state[q]["step"] = n.clone()

    def pending(self) -> bool:
        return bool(self.queue)

    def drain_to(self, pipeline) -> None:
        """Mode switch with batches fetched: hand them back to the generic pipeline in order."""
        from .torchrec.distributed.train_pipeline import _Staged

        items, self.queue = self.queue, []
        self._reset()
        if items:
            pipeline._cur = _Staged(items[0].batch, None)
            pipeline._next = _Staged(items[1].batch, None) if len(items) > 1 else None
            pipeline._pushback = [x.batch for x in items[2:]] + list(getattr(pipeline, "_pushback", []))

    # ---- one progress() ----------------------------------------------------------------------
    def progress(self, it: Iterator) -> Any:
        self._fill(it)
        if not self.queue:
            self._reset()
            self.check_errors()
            self.sync_optimizer_state()
            raise StopIteration
        cur = self.queue[0]
        if cur.slot is None:
            self._reset()
            out = self._generic(cur.batch)
        else:
            out = self._fused()
        self.queue.pop(0)
        return out

    def _fused(self) -> Any:
        st = self.step
        q = self.queue
        cur = q[0]
        nxt = q[1] if len(q) > 1 and q[1].slot is not None else None
        nxt2 = q[2] if nxt is not None and len(q) > 2 and q[2].slot is not None else None
        lr = self._group["lr"]
        if lr != st.lr_dense:  # the plans carry Adam's lr: re-capture after a change
            st.lr_dense = float(lr)
            if self.graph_mode:
                self._capture()
        if not self.staged:
            st.prime(self.slot_cols[cur.slot], cur.parity,
                     self.slot_cols[nxt.slot] if nxt is not None else self.zero_cols)
        if self.graph_mode and nxt2 is not None and nxt2.slot == (cur.slot + 2) % self.depth:
            self.graphs[cur.slot].replay()
        else:
            self._pipelined(cur.slot, cur.parity, self.slot_cols[nxt2.slot] if nxt2 is not None else self.zero_cols)
        self.staged = nxt is not None
        self.dirty = True
        self.steps_fused += 1
        return self.slot_loss[cur.slot], self.slot_logits[cur.slot], cur.labels

    def _generic(self, batch) -> Any:
        """A batch the fused step does not take: the DMP per-op path (collective on every rank),
        the Adam step count carried across (the moments are shared views)."""
        p = self.pipeline
        st = self.step
        if st is not None:
            n = int(st.adam_state[0].item())
            for q in self._params:
                self.adam.state[q]["step"] = torch.tensor(float(n))
        p._optimizer.zero_grad(set_to_none=True)
        losses, output = p._model(batch)
        torch.sum(losses, dim=0).backward()
        p._optimizer.step()
        if st is not None:
            st.adam_state[0] = n + 1
            st.towers.update(st.params, do_adam=False)
        self.steps_generic += 1
        return output
