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

At world size W > 1 (DistributedModelParallel over W processes) ``FusedShardedDropin`` below takes the
loop instead: the pipelined sharded step for single-hot bags, the sharded KJT step for multi-hot
bags, each batch admitted by every rank (an agreed per-batch check) or run through the generic DMP
path on every rank. Conditions at world size 1 (else the generic per-op path runs, unchanged):
``TwoTowerTrainTask(TwoTower)`` with one feature per tower, equal embedding dims of
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
    __slots__ = ("batch", "slot", "parity", "labels", "primed", "seq", "adm", "event", "work", "agreed")

    def __init__(self, batch, slot=None, parity=0, labels=None):
        self.batch = batch
        self.slot = slot
        self.parity = parity
        self.labels = labels
        self.primed = False
        self.seq = -1
        self.adm = None      # N > 1: this rank's admission vector (pinned int64) / the agreed one
        self.event = None    # N > 1: the admission counts have reached the host
        self.work = None     # N > 1: the async all-reduce of the admission vector
        self.agreed = None   # N > 1: the MAX over the ranks (numpy), once known


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




# The N > 1 drop-in's admission vector of one batch (int64), MAX-reduced over the ranks before the
# batch trains on a fused sharded step: every rank then takes the same path for it, whatever its own
# data looked like (a mismatch would run different collectives on different ranks).
A_REJECT, A_B, A_NEGB, A_DT, A_NEGDT, A_MULTI, A_OVER, A_ERR, A_SEG, A_DEST, A_NNZ = range(11)
A_LEN = 12
_RING = 16  # admission count buffers in flight (fetched, not yet on the host)


class FusedShardedDropin:
    """The reference's loop at world size W > 1 (DistributedModelParallel over W processes, one GPU
    each, 03_model_training.py:812-815, :918) on the fused sharded steps: TrainPipelineSparseDist.progress
    hands each batch to a step that trains the ShardedEmbeddingBagCollection's OWN shards (table-wise or
    row-wise per the DMP plan; ``ops.TableSet.view_of``) and the towers' parameters and Adam moments as
    views of its flat buffers (the DDP replicas: the step's fixed-order mean of the W tower gradients is
    DDP's all-reduce mean). Fixed-size exchanges (device-initiated into the peers' buffers after
    ``sharded.exchange_comm``'s self-test, else RCCL) instead of the eager input_dist / output_dist /
    DDP collectives with their host-synchronised split sizes (torchrec/distributed/embeddingbag.py).

    Two modes, fixed by the first batch every rank admits:
      "pipelined"  single-hot bags: ``sharded.FusedShardedTwoTowerStep``, two batches of lookahead
                   (batch i+1's rows gathered during step i, batch i+2's ids routed), one HIP graph per
                   slot; a multi-hot batch later runs the generic DMP path;
      "kjt"        multi-hot bags (BASELINE config 5): ``sharded_kjt.FusedShardedKJTStep``, three
                   exchanges per batch (ids in, one pooled row per (bag, owner) out, bag gradients
                   back), one HIP graph per slot; any bag lengths.

    Admission. Every fetched batch gets an admission vector (``tt_kjt_admit`` on a side stream: bags
    longer than one id, values outside [0, N), ids per (owner, feature) segment; plus batch size, id
    dtype, value count and this rank's own shape checks), MAX-reduced over the ranks by an async
    all-reduce on a gloo group of the same ranks (issued in fetch order, typically two progress calls
    before it is needed). A batch trains fused only if EVERY rank admits it: same batch size and id
    dtype, no value out of range, no segment over its capacity (the capacities come from the first
    batch: its largest segment x 1.5), single-hot in the pipelined mode. Anything else — a smaller
    last batch, a skewed batch beyond a capacity, a multi-id bag in the pipelined mode — runs the
    generic DMP path on every rank between fused steps (the staged pipeline dropped first; a route
    that overflowed only ever belonged to such a batch, so no fused step trains on dropped lookups).
    ``TT_DROPIN_EXCHANGE`` = auto (default) / peer / rccl picks the exchange."""

    def __init__(self, pipeline, task, ebc, ts, fused_cfg, towers, adam, feats, dims, sharded, depth: int = 8):
        import ctypes as C

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
        self.W = W = dist.get_world_size(ebc._pg)
        self.N = [c.num_embeddings for c in ebc._embedding_bag_configs]
        self.blocks = [-(-n // W) if s == "row_wise" else 0 for n, s in zip(self.N, self.sharding)]
        self.seg_owner = [o if s == "table_wise" else 0 for o, s in zip(self.owners, self.sharding)]
        self.mode = None  # "pipelined" | "kjt", fixed by the first admitted batch
        self.step = None
        self.comm = None
        self.exchange = ""
        self.queue: List[_Item] = []  # fetched batches: cur, nxt, nxt2
        self.staged = False  # pipelined: the step holds batch queue[0]'s rows and the next batch's route
        self.dirty = False   # pipelined: a fused step ran since the last reset (its dedup tables hold keys)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)  # the conversion's word (unused:
        # the admission vector carries the same facts per batch)
        self.steps_fused = 0
        self.steps_generic = 0
        self.rejected = {}  # reason -> batches sent down the generic path by the agreed admission
        self.graphs: List = []
        self.graph_mode = None
        self.lr_captured = None
        # admission: counts on a side stream, agreement over a gloo group of the same ranks
        self._apg = dist.new_group(ranks=dist.get_process_group_ranks(ebc._pg), backend="gloo")
        self._astream = torch.cuda.Stream(device=self.device)
        self._aout = [torch.zeros(2 + W * 2, dtype=torch.int32, device=self.device) for _ in range(_RING)]
        self._ahost = [torch.zeros(2 + W * 2, dtype=torch.int32).pin_memory() for _ in range(_RING)]
        self._pending: List[_Item] = []  # admission vectors not yet reduced, in fetch order
        self._works: List[_Item] = []    # reductions issued, not yet waited on
        self._seq = 0
        self._lib = _lib.load()
        self._ne = (C.c_int64 * 2)(*self.N)
        self._bs = (C.c_int64 * 2)(*self.blocks)
        self._ow = (C.c_int32 * 2)(*self.seg_owner)

    # reuse of the single-GPU drop-in's helpers
    _adam_group = FusedDropin._adam_group
    _adam_lr = FusedDropin._adam_lr

    # ---- admission ---------------------------------------------------------------------------
    def _local_ok(self, batch) -> bool:
        """This rank's own shape checks (the agreed admission adds everything that needs all ranks)."""
        kjt = getattr(batch, "sparse_features", None)
        if kjt is None or list(kjt.keys()) != self.feats:
            return False
        B = kjt.stride()
        if B < 8 or B % 8 or (self.step is not None and B != self.step.B):
            return False
        v = kjt.values()
        if v.numel() and v.dtype not in (torch.int32, torch.int64):
            return False
        if self.step is not None and v.numel() and v.dtype != self.id_dtype:
            return False
        if self.mode == "kjt" and v.numel() > self.vcap:
            return False
        lab = batch.labels
        return (lab.numel() == B and lab.dtype in (torch.int32, torch.int64) and lab.is_contiguous()
                and lab.device == self.device and kjt.device() == self.device)

    @staticmethod
    def _offsets32(kjt) -> torch.Tensor:
        o = kjt.offsets()
        return o if o.dtype == torch.int32 else o.to(torch.int32)

    def _counts(self, batch, offs, out, stream) -> None:
        kjt = batch.sparse_features
        v = kjt.values()
        idt = _lib.id_dtype_code(v.dtype) if v.numel() else _lib.TT_I64
        _lib.check(self._lib.tt_kjt_admit(2, kjt.stride(), v.data_ptr() if v.numel() else None, idt, v.numel(),
                                          offs.data_ptr(), self._ne, self._bs, self._ow, self.W, out.data_ptr(),
                                          stream.cuda_stream), "kjt_admit")

    def _vector(self, ok: bool, batch, counts: Optional[torch.Tensor]) -> torch.Tensor:
        """This rank's admission vector (host int64) from its shape checks and the batch's counts."""
        import numpy as np

        a = np.zeros(A_LEN, dtype=np.int64)
        kjt = getattr(batch, "sparse_features", None)
        B = kjt.stride() if kjt is not None else 0
        a[A_B], a[A_NEGB] = B, -B
        a[A_REJECT] = 0 if ok else 1
        if ok:
            v = kjt.values()
            dt = 1 if (v.dtype == torch.int64 if v.numel() else (self.id_dtype == torch.int64 if self.step else True)) \
                else 0
            a[A_DT], a[A_NEGDT] = dt, -dt
            c = counts.numpy().astype(np.int64)
            cnt = c[2:].reshape(self.W, 2)
            a[A_MULTI] = 1 if c[0] else 0
            a[A_ERR] = c[1]
            rw = [f for f in range(2) if self.sharding[f] == "row_wise"]
            a[A_SEG] = int(cnt[:, rw].max()) if rw else 0
            a[A_DEST] = int(cnt.sum(axis=1).max())
            a[A_NNZ] = v.numel()
            if self.step is not None:
                if self.mode == "pipelined":
                    a[A_OVER] = int(any(cnt[d, f] > self.step.caps_f[f] for d in range(self.W) for f in rw))
                else:
                    a[A_OVER] = int(a[A_DEST] > self.step.cap)
        return torch.from_numpy(a)

    def _reason(self, ag, first: bool = False) -> str:
        """'' if every rank admits the batch (agreed vector ``ag``), else why not."""
        if ag[A_REJECT]:
            return "a rank's batch is not the step's shape (keys, batch size, dtypes, value capacity)"
        if ag[A_B] != -ag[A_NEGB]:
            return "the ranks' batch sizes differ"
        if ag[A_DT] != -ag[A_NEGDT]:
            return "the ranks' id dtypes differ"
        if ag[A_ERR]:
            return "an id outside [0, N)"
        if not first and ag[A_OVER]:
            return "a segment over its capacity (skewed ids)"
        if not first and self.mode == "pipelined" and ag[A_MULTI]:
            return "a bag of several ids (the single-hot pipelined step)"
        return ""

    def _poll(self, upto: int = -1) -> None:
        """Issue the agreement of every fetched batch whose counts reached the host, in fetch order
        (forcing those up to sequence number ``upto``)."""
        import torch.distributed as dist

        while self._pending:
            x = self._pending[0]
            if x.event is not None:
                if not x.event.query():
                    if x.seq > upto:
                        break
                    x.event.synchronize()
                x.adm = self._vector(True, x.batch, x.adm)
                x.event = None
            x.work = dist.all_reduce(x.adm, op=dist.ReduceOp.MAX, group=self._apg, async_op=True)
            self._works.append(x)
            self._pending.pop(0)

    def _agreed(self, x: _Item):
        if x.agreed is None:
            self._poll(upto=x.seq)
            x.work.wait()
            x.agreed = x.adm.numpy().copy()
            self._works = [w for w in self._works if w is not x]
        return x.agreed

    def _settle(self) -> None:
        """Every fetched batch's agreement issued and completed (before the pipeline hands batches back
        or ends: every rank reduces every batch it fetched)."""
        self._poll(upto=self._seq)
        for x in self._works:
            x.work.wait()
            if x.agreed is None:
                x.agreed = x.adm.numpy().copy()
        self._works = []

    def _admit_first(self, batch, ok: bool, offs) -> Tuple[bool, Any]:
        """The first batch(es), before any step exists: counted and agreed synchronously (every rank
        reaches this with the same batch index)."""
        import torch.distributed as dist

        counts = None
        if ok:
            out = self._aout[0]
            self._counts(batch, offs, out, torch.cuda.current_stream(self.device))
            counts = out.cpu()
        a = self._vector(ok, batch, counts)
        dist.all_reduce(a, op=dist.ReduceOp.MAX, group=self._apg)
        ag = a.numpy().copy()
        why = self._reason(ag, first=True)
        return not why, ag

    # ---- the steps on the sharded EBC's storage -------------------------------------------------
    def _adopt_towers(self, st) -> None:
        """The towers' parameters -> views of the step's flat buffer; Adam's moments likewise."""
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

    def _make_step(self, batch, ag) -> None:
        import ctypes as C

        import torch.distributed as dist

        from .sharded import PeerComm, default_capacity, exchange_comm
        from .sharded_kjt import FusedShardedKJTStep

        kjt = batch.sparse_features
        B = kjt.stride()
        self.id_dtype = idt = torch.int64 if ag[A_DT] else torch.int32
        dev, W, ebc, D = self.device, self.W, self.ebc, self.dims[0]
        self.mode = "kjt" if ag[A_MULTI] else "pipelined"
        local = [ebc._local_index.get(ebc._f_table[f]) for f in range(2)]
        tables = ops.TableSet.view_of(self.ts, local, [D, D], dev)
        self.comm, self.exchange = exchange_comm(os.environ.get("TT_DROPIN_EXCHANGE", "auto"), group=ebc._pg,
                                                 device=dev)
        kw = dict(lr_emb=self.fused_cfg["lr"], lr_dense=self._adam_lr(), eps=self.fused_cfg["eps"], tables=tables)
        if self.mode == "pipelined":
            from .sharded import FusedShardedTwoTowerStep

            cap = max(default_capacity(B, W, factor=1.5), -(-int(ag[A_SEG]) * 3 // 2))
            cap = min(B, -(-cap // 8) * 8)
            st = FusedShardedTwoTowerStep(self.comm, self.N, D, [128, 64], B, dev, sharding=self.sharding,
                                          tw_owners=self.owners, id_dtype=idt, capacity=cap, **kw)
        else:
            cap = max(64, -(-int(ag[A_DEST]) * 3 // 2))
            cap = -(-cap // 8) * 8
            st = FusedShardedKJTStep(self.comm, self.N, D, [128, 64], B, dev, cap, sharding=self.sharding,
                                     tw_owners=self.owners, **kw)
        self._adopt_towers(st)
        self.step = st
        Dp = self.depth
        self.slot_labels = [torch.zeros(B, dtype=torch.int32, device=dev) for _ in range(Dp)]
        self.slot_logits = [torch.zeros(B, dtype=torch.float32, device=dev) for _ in range(Dp)]
        self.slot_loss = [torch.zeros((), dtype=torch.float32, device=dev) for _ in range(Dp)]
        if self.mode == "pipelined":
            self.slot_cols = [[torch.zeros(B, dtype=idt, device=dev) for _ in range(2)] for _ in range(Dp)]
            self.zero_cols = [torch.zeros(B, dtype=idt, device=dev) for _ in range(2)]
            self._slot_ptrs = [_lib.ptr_array(c) for c in self.slot_cols]
        else:
            # values capacity per slot: twice the largest first batch (a larger batch: generic path)
            self.vcap = max(2 * int(ag[A_NNZ]), 2 * B)
            self.slot_values = [torch.zeros(self.vcap, dtype=idt, device=dev) for _ in range(Dp)]
            self.slot_offsets = [torch.zeros(2 * B + 1, dtype=torch.int32, device=dev) for _ in range(Dp)]
        self._ne2 = (C.c_int64 * 2)(*self.N)
        self._idt = _lib.id_dtype_code(idt)
        self._group = self._adam_group()
        # graphs with the collectives inside: the device-initiated exchange (any backend) or RCCL
        self.graph_mode = isinstance(self.comm, PeerComm) or dist.get_backend(ebc._pg) == "nccl"
        if self.graph_mode:
            try:
                self._capture()
            except Exception as e:  # noqa: BLE001 - the same collectives run eagerly
                import sys

                print(f"dropin (sharded): graph capture refused ({e}); eager steps", file=sys.stderr)
                torch.cuda.synchronize(dev)
                self.graphs, self.graph_mode = [], False
                if self.mode == "pipelined":
                    st.reset_pipeline()
        if self.mode == "kjt":
            st.cursor = 0

    def _kjt_step(self, slot: int) -> None:
        st = self.step
        keep = st.logits, st.loss
        st.logits, st.loss = self.slot_logits[slot], self.slot_loss[slot]
        try:
            st.step(self.slot_values[slot], self.slot_offsets[slot], self.slot_labels[slot])
        finally:
            st.logits, st.loss = keep

    def _pipelined(self, slot: int, parity: int, next2) -> None:
        st = self.step
        keep = st.logits, st.loss
        st.logits, st.loss = self.slot_logits[slot], self.slot_loss[slot]
        try:
            st.step_pipelined(self.slot_labels[slot], parity, next2)
        finally:
            st.logits, st.loss = keep

    def _capture(self) -> None:
        """Slot k's graph: pipelined, the step on slot k (parity k % 2) routing slot k + 2; kjt, the
        step on slot k's batch."""
        st, Dp, dev = self.step, self.depth, self.device
        self.lr_captured = st.lr_dense
        if self.mode == "kjt" and not self.graphs:
            st.warmup()  # communicators, workspaces (the training state is left as it was)
        st.comm.retire()
        self.graphs = []
        torch.cuda.synchronize(dev)
        for k in range(Dp):
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    if self.mode == "kjt":
                        self._kjt_step(k)
                    else:
                        self._pipelined(k, k % 2, self.slot_cols[(k + 2) % Dp])
            torch.cuda.current_stream(dev).wait_stream(s)
            _lib.graph_upload(g, dev)
            self.graphs.append(g)
        torch.cuda.synchronize(dev)

    # ---- staging -----------------------------------------------------------------------------
    def _stage(self, x: _Item, batch, offs) -> None:
        """The batch into slot seq % depth (main stream): pipelined, its single-hot ids as id columns
        (tt_kjt_single_hot_cols); kjt, its values / offsets copied; labels as int32."""
        kjt = batch.sparse_features
        v = kjt.values()
        slot = x.seq % self.depth
        lab = batch.labels
        stream = torch.cuda.current_stream(self.device)
        if self.mode == "pipelined":
            _lib.check(self._lib.tt_kjt_single_hot_cols(
                2, self.step.B, v.data_ptr() if v.numel() else self.slot_cols[slot][0].data_ptr(), self._idt,
                offs.data_ptr(), self._ne2, self._slot_ptrs[slot], self.err.data_ptr(), lab.data_ptr(),
                _lib.TT_I64 if lab.dtype == torch.int64 else _lib.TT_I32, self.slot_labels[slot].data_ptr(),
                stream.cuda_stream), "kjt_single_hot_cols")
        else:
            if v.numel():
                self.slot_values[slot][:v.numel()].copy_(v, non_blocking=True)
            self.slot_offsets[slot].copy_(offs, non_blocking=True)
            self.slot_labels[slot].copy_(lab, non_blocking=True)
        x.slot, x.parity, x.labels = slot, x.seq % 2, lab

    def _fetch(self, it: Iterator) -> Optional[_Item]:
        try:
            batch = next(it)
        except StopIteration:
            return None
        batch = batch.to(self.device, non_blocking=True)
        x = _Item(batch)
        x.seq = self._seq
        self._seq += 1
        ok = self._local_ok(batch)
        offs = self._offsets32(batch.sparse_features) if ok else None
        if self.step is None:
            adm, ag = self._admit_first(batch, ok, offs)
            x.agreed = ag
            if not adm:
                self._note(self._reason(ag, first=True))
                return x
            self._make_step(batch, ag)
            self._stage(x, batch, offs)
            return x
        if ok:
            j = x.seq % _RING
            main = torch.cuda.current_stream(self.device)
            ev0 = torch.cuda.Event()
            ev0.record(main)
            with torch.cuda.stream(self._astream):
                self._astream.wait_event(ev0)
                self._counts(batch, offs, self._aout[j], self._astream)
                self._ahost[j].copy_(self._aout[j], non_blocking=True)
                x.event = torch.cuda.Event()
                x.event.record(self._astream)
            offs.record_stream(self._astream)
            batch.sparse_features.values().record_stream(self._astream)
            x.adm = self._ahost[j]  # the counts until _poll turns them into the vector
            self._stage(x, batch, offs)
        else:
            x.adm = self._vector(False, batch, None)
        self._pending.append(x)
        return x

    def _fill(self, it: Iterator) -> None:
        while len(self.queue) < 3:
            x = self._fetch(it)
            if x is None:
                break
            self.queue.append(x)

    def _note(self, why: str) -> None:
        if why:
            self.rejected[why] = self.rejected.get(why, 0) + 1

    def _reset(self) -> None:
        if self.mode == "pipelined" and self.step is not None and self.dirty:
            self.step.reset_pipeline()
        self.staged = self.dirty = False

    def check_errors(self) -> None:
        """Raise (on every rank) if a step received a key outside its shard or a device-initiated
        exchange timed out (collective). Multi-id bags, ids out of range and segment overflows never
        reach a fused step (the agreed admission sends such batches down the generic path)."""
        if self.step is not None:
            self.step.check()

    def sync_optimizer_state(self) -> None:
        if self.step is None:
            return
        n = torch.tensor(float(int(self.step.adam_state[0].item())))
        for q in self._params:
            self.adam.state[q]["step"] = n.clone()

    def pending(self) -> bool:
        return bool(self.queue)

    def drain_to(self, pipeline) -> None:
        """Mode switch with batches fetched: hand them back to the generic pipeline in order (their
        agreements completed first: every rank reduced every batch it fetched)."""
        from .torchrec.distributed.train_pipeline import _Staged

        self._settle()
        items, self.queue = self.queue, []
        self._reset()
        if items:
            pipeline._cur = _Staged(items[0].batch, None)
            pipeline._next = _Staged(items[1].batch, None) if len(items) > 1 else None
            pipeline._pushback = [x.batch for x in items[2:]] + list(getattr(pipeline, "_pushback", []))

    # ---- one progress() ----------------------------------------------------------------------
    def progress(self, it: Iterator) -> Any:
        self._fill(it)
        self._poll()
        if not self.queue:
            self._settle()
            self._reset()
            self.check_errors()
            self.sync_optimizer_state()
            raise StopIteration
        cur = self.queue[0]
        if cur.slot is not None and self.step is not None:
            why = self._reason(self._agreed(cur))
            if why:  # some rank cannot run it fused: every rank runs it through the generic path
                self._note(why)
                cur.slot = None
                if self.mode == "pipelined":
                    self.step.flags[0:1].zero_()  # an overflow of THIS batch's route (dropped lookups, untrained)
        if cur.slot is None:
            self._reset()
            out = self._generic(cur.batch)
        elif self.mode == "kjt":
            out = self._fused_kjt(cur)
        else:
            out = self._fused()
        self.queue.pop(0)
        return out

    def _relr(self) -> None:
        lr = self._group["lr"]
        if lr != self.step.lr_dense:  # the plans carry Adam's lr: re-capture after a change
            self.step.lr_dense = float(lr)
            if self.graph_mode:
                if self.mode == "pipelined" and self.dirty:
                    self.step.reset_pipeline()
                    self.staged = self.dirty = False
                self._capture()

    def _fused_kjt(self, cur: _Item) -> Any:
        self._relr()
        if self.graph_mode:
            self.graphs[cur.slot].replay()
        else:
            self._kjt_step(cur.slot)
        self.steps_fused += 1
        return self.slot_loss[cur.slot], self.slot_logits[cur.slot], cur.labels

    def _fused(self) -> Any:
        st = self.step
        q = self.queue
        cur = q[0]
        nxt = q[1] if len(q) > 1 and q[1].slot is not None else None
        nxt2 = q[2] if nxt is not None and len(q) > 2 and q[2].slot is not None else None
        self._relr()
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
