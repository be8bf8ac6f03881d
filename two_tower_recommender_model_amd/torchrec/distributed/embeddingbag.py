"""Sharded EmbeddingBagCollection (torchrec.distributed.embeddingbag) for one process per MI355X.

Built by DistributedModelParallel (03_model_training.py:812-815) from the plan's ParameterShardings:

  TABLE_WISE  table t lives whole on rank owner(t).
  ROW_WISE    table t is split into contiguous row blocks of bs = ceil(N/W); rank p holds rows
              [p*bs, (p+1)*bs) (block_bucketize semantics).

One forward, per rank (local batch B, W ranks):
  input_dist   KJT.permute -> (TW) keys grouped by owner; (RW) block_bucketize -> bucket-major ids.
               1 tiny all-to-all of per-peer counts, then ONE all-to-all of lengths and ONE of
               ids, each packing the TW and RW parts for a peer together.
  lookup       the received ids form a local KJT whose keys are (source rank s, feature k); one
               tt_pooled_fwd launch per sharding group writes source s's bags at rows s*B..s*B+B.
  output_dist  TW: all-to-all of pooled rows back to their source ranks; RW: reduce-scatter of the
               [W*B, D] partial sums (torchrec's RW semantics), then the columns are placed in
               KeyedTensor (EBC feature) order.
Backward: the adjoint collectives (TW all-to-all back, RW all-gather) and the fused dedup +
row-wise Adagrad kernels on the local shards. The dense towers stay replicated under DDP.

Collectives go through torch.distributed: "nccl" = RCCL over xGMI on the GPU box; the same code
runs on "gloo" over CPU for the multi-process tests (with a test-provided lookup backend).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from torch import nn

from ... import _lib, ops
from ..modules.embedding_modules import EmbeddingBagCollection, _fused_config, _TableModule
from ..sparse.jagged_tensor import KeyedJaggedTensor, KeyedTensor
from .types import ParameterSharding, ShardingType


class EmbeddingBagCollectionSharder:
    """torchrec.distributed.embeddingbag.EmbeddingBagCollectionSharder (get_default_sharders())."""

    def __init__(self, fused_params: Optional[dict] = None, qcomm_codecs_registry=None, lookup_backend=None):
        """lookup_backend: the local lookup of the sharded modules this sharder builds (None = the
        HIP kernels, ops.HIP_BACKEND; the multi-process CPU tests pass their oracle-backed one)."""
        self.fused_params = fused_params or {}
        self.lookup_backend = lookup_backend

    def sharding_types(self, compute_device_type: str) -> List[str]:
        return [ShardingType.TABLE_WISE.value, ShardingType.ROW_WISE.value]

    def compute_kernels(self, sharding_type: str, compute_device_type: str) -> List[str]:
        return ["fused"]

    @property
    def module_type(self):
        return EmbeddingBagCollection


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits: List[int], in_splits: List[int], pg) -> None:
    dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits, group=pg)


def _reduce_scatter_rows(out: torch.Tensor, inp: torch.Tensor, W: int, pg) -> None:
    """out[B, D] = sum over ranks of their inp[rank*B:(rank+1)*B] (reduce-scatter along dim 0)."""
    if dist.get_backend(pg) == "gloo":
        recv = torch.empty((W,) + tuple(out.shape), dtype=out.dtype, device=out.device)
        dist.all_to_all_single(recv, inp.contiguous(), group=pg)
        torch.sum(recv, dim=0, out=out)
    else:
        dist.reduce_scatter_tensor(out, inp.contiguous(), group=pg)


def _all_gather_rows(out: torch.Tensor, inp: torch.Tensor, pg) -> None:
    """out[W*B, D] = every rank's inp[B, D], rank-major (all-gather along dim 0)."""
    if dist.get_backend(pg) == "gloo" and inp.is_cuda:
        # gloo (the CPU tests and the one-GPU multi-process rehearsal): its all-to-all takes device
        # tensors, so the all-gather is an all-to-all of the input repeated for every destination
        W = dist.get_world_size(pg)
        dist.all_to_all_single(out, inp.contiguous().repeat(W, 1), group=pg)
    else:
        dist.all_gather_into_tensor(out, inp.contiguous(), group=pg)


class _ShardedLookup(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, dist_ctx, *params):
        kt_values, saved = mod._lookup_output_dist(dist_ctx)
        ctx.mod = mod
        ctx.saved = saved
        return kt_values

    @staticmethod
    def backward(ctx, grad):
        ctx.mod._backward_impl(grad, ctx.saved)
        return (None, None) + (None,) * len(ctx.mod._local_params())


def _sharded_state_dict_hook(module, state_dict, prefix, local_metadata):
    """state_dict() of a sharded EBC holds one torch ShardedTensor per table (collective: every rank
    builds every table's, with no local shard where it holds none), as torchrec's does — what the
    reference's gather_and_get_state_dict (03_model_training.py:474-495) expects:
    ``isinstance(t, ShardedTensor)`` then ``t.gather(0, full)`` on rank 0."""
    from torch.distributed._shard.metadata import ShardMetadata
    from torch.distributed._shard.sharded_tensor import Shard, ShardedTensor

    dev = module._device
    place = f"rank:{module._rank}/{dev.type}" + (f":{dev.index if dev.index is not None else 0}"
                                                 if dev.type == "cuda" else "")
    for c in module._embedding_bag_configs:  # same key order on every rank (collective gathers follow it)
        state_dict.pop(f"{prefix}embedding_bags.{c.name}.weight", None)
    for t, c in enumerate(module._embedding_bag_configs):
        key = f"{prefix}embedding_bags.{c.name}.weight"
        shards = []
        lo, n = module._shard_of.get(t, (0, 0))
        if n > 0:
            w = module.embedding_bags[c.name].weight.detach()
            shards.append(Shard(tensor=w, metadata=ShardMetadata(shard_offsets=[lo, 0],
                                                                 shard_sizes=[n, c.embedding_dim],
                                                                 placement=place)))
        state_dict[key] = ShardedTensor._init_from_local_shards(shards, c.num_embeddings, c.embedding_dim,
                                                                process_group=module._pg)
    state_dict.pop(prefix + "_grad_anchor", None)
    return state_dict


def _sharded_load_pre_hook(module, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                           error_msgs):
    """load_state_dict() of a sharded EBC takes full (gathered) tables: each rank keeps its rows."""
    for t, c in enumerate(module._embedding_bag_configs):
        key = f"{prefix}embedding_bags.{c.name}.weight"
        if key not in state_dict:
            continue
        full = state_dict.pop(key)
        if c.name in module.embedding_bags:  # this rank's rows replace the full table
            lo, n = module._shard_of.get(t, (0, 0))
            state_dict[key] = full[lo:lo + n]
    state_dict.setdefault(prefix + "_grad_anchor", module._grad_anchor.detach())


class ShardedEmbeddingBagCollection(nn.Module):
    def __init__(self, ebc: EmbeddingBagCollection, module_plan: Dict[str, ParameterSharding], pg,
                 device: torch.device, backend=None):
        super().__init__()
        self._pg = pg
        self._W = dist.get_world_size(pg)
        self._rank = dist.get_rank(pg)
        self._device = torch.device(device)
        self._be = backend or ops.HIP_BACKEND
        self._embedding_bag_configs = ebc.embedding_bag_configs()
        self._pooling = ebc._pooling
        self._fused = _fused_config(ebc._params())
        if self._fused is None:
            raise NotImplementedError(
                "sharded tables need the fused in-backward optimizer: call "
                "_apply_optimizer_in_backward(RowWiseAdagrad, ebc.parameters(), {'lr': ...}) before DMP")
        cfgs = self._embedding_bag_configs
        W, r = self._W, self._rank
        self._feature_names = list(ebc._feature_names)
        self._dims = list(ebc._lengths_per_embedding)
        f_table = list(ebc._feature_table)
        col = [0]
        for d in self._dims:
            col.append(col[-1] + d)
        self._cols = col
        self._out_dim = col[-1]
        shard = {}
        for t, c in enumerate(cfgs):
            ps = module_plan.get(c.name)
            if ps is None:
                raise ValueError(f"no sharding for table {c.name}")
            shard[t] = ps
        self._plan = module_plan
        # ---- groups
        self._tw_feats = [f for f in range(len(f_table)) if shard[f_table[f]].sharding_type == ShardingType.TABLE_WISE.value]
        self._rw_feats = [f for f in range(len(f_table)) if shard[f_table[f]].sharding_type == ShardingType.ROW_WISE.value]
        other = [f for f in range(len(f_table)) if f not in self._tw_feats and f not in self._rw_feats]
        if other:
            raise NotImplementedError("only TABLE_WISE / ROW_WISE shardings are supported")
        owner = {t: shard[t].ranks[0] for t in range(len(cfgs)) if shard[t].sharding_type == ShardingType.TABLE_WISE.value}
        self._tw_by_owner = [[f for f in self._tw_feats if owner[f_table[f]] == o] for o in range(W)]
        self._tw_order = [f for o in range(W) for f in self._tw_by_owner[o]]
        # ---- local storage: TW tables owned here + this rank's block of every RW table
        local_tables: List[Tuple[int, int, int]] = []  # (table idx, row_lo, rows)
        for t, c in enumerate(cfgs):
            if shard[t].sharding_type == ShardingType.TABLE_WISE.value and owner[t] == r:
                local_tables.append((t, 0, c.num_embeddings))
        self._rw_block = {}
        for t, c in enumerate(cfgs):
            if shard[t].sharding_type == ShardingType.ROW_WISE.value:
                bs = (c.num_embeddings + W - 1) // W
                lo = min(r * bs, c.num_embeddings)
                n = max(0, min(bs, c.num_embeddings - lo))
                self._rw_block[t] = bs
                local_tables.append((t, lo, n))
        self._local_tables = local_tables
        self._local_index = {t: i for i, (t, _, _) in enumerate(local_tables)}
        self.embedding_bags = nn.ModuleDict()
        self._ts = None
        if local_tables:
            rows = [max(1, n) for (_, _, n) in local_tables]
            dims = [cfgs[t].embedding_dim for (t, _, _) in local_tables]
            self._ts = self._be.table_set(rows, dims, [0], self._device)
            old = {c.name: ebc.embedding_bags[c.name].weight for c in cfgs if c.name in ebc.embedding_bags}
            for i, (t, lo, n) in enumerate(local_tables):
                c = cfgs[t]
                view = self._ts.table_view(i)
                src = old.get(c.name)
                if src is not None and src.device.type != "meta":
                    view[:n].copy_(src.detach()[lo:lo + n])
                else:
                    view.uniform_(c.get_weight_init_min(), c.get_weight_init_max())
                self.embedding_bags[c.name] = _TableModule(nn.Parameter(view[:n]))
        # feature index maps
        self._tw_me = self._tw_by_owner[r]
        self._tw_me_cols = self._prefix([self._dims[f] for f in self._tw_me])
        self._rw_cols_local = self._prefix([self._dims[f] for f in self._rw_feats])
        self._f_table = f_table
        self._ts_cache: Dict[Tuple[str, int], object] = {}
        self._grad_anchor = nn.Parameter(torch.zeros(0, device=self._device))
        # input_dist results staged by TrainPipelineSparseDist: [(kjt, dist ctx)], newest last, matched
        # by the KJT object's identity (not id(): a freed KJT's id is reused), at most two kept
        self._prefetched: List[Tuple[KeyedJaggedTensor, dict]] = []
        self._shard_of = {t: (lo, n) for (t, lo, n) in local_tables}
        self._register_state_dict_hook(_sharded_state_dict_hook)
        self._register_load_state_dict_pre_hook(_sharded_load_pre_hook, with_module=True)

    @staticmethod
    def _prefix(ds: Sequence[int]) -> List[int]:
        out, o = [], 0
        for d in ds:
            out.append(o)
            o += d
        return out

    # -- torchrec API
    def embedding_bag_configs(self):
        return self._embedding_bag_configs

    def _local_params(self):
        return [self._grad_anchor]

    def _lookup_ts(self, group: str, Bm: int):
        """TableSet view whose keys are (source rank s, feature k) of the group, bags of s at rows s*Bm."""
        key = (group, Bm)
        ts = self._ts_cache.get(key)
        if ts is None:
            feats = self._tw_me if group == "tw" else self._rw_feats
            cols = self._tw_me_cols if group == "tw" else self._rw_cols_local
            ft, oo, orow = [], [], []
            for s in range(self._W):
                for j, f in enumerate(feats):
                    ft.append(self._local_index[self._f_table[f]])
                    oo.append(cols[j])
                    orow.append(s * Bm)
            ts = self._ts.remap(ft, oo, orow)
            self._ts_cache[key] = ts
        return ts

    # -- forward
    def forward(self, features: KeyedJaggedTensor) -> KeyedTensor:
        d = None
        for i, (k, staged) in enumerate(self._prefetched):
            if k is features:
                d = staged
                del self._prefetched[i]
                break
        if d is None:
            d = self.input_dist(features)
        elif d["stream"] is not None:  # staged by TrainPipelineSparseDist on its data-dist stream
            cur = torch.cuda.current_stream(self._device)
            cur.wait_event(d["event"])
            for t in d["tensors"]:
                t.record_stream(cur)
        vals = _ShardedLookup.apply(self, d, self._grad_anchor)
        return KeyedTensor(self._feature_names, self._dims, vals)

    def prefetch(self, features: KeyedJaggedTensor) -> None:
        """input_dist of a batch ahead of its forward (TrainPipelineSparseDist's second stage), on the
        current stream; ``forward(features)`` of the same KJT object then consumes it."""
        d = self.input_dist(features)
        if torch.cuda.is_available() and self._device.type == "cuda":
            s = torch.cuda.current_stream(self._device)
            d["stream"] = s
            d["event"] = torch.cuda.Event()
            d["event"].record(s)
        self._prefetched.append((features, d))
        del self._prefetched[:-2]  # a batch whose forward never ran (an exception, a derived KJT)

    def accepts(self, features: KeyedJaggedTensor) -> bool:
        """Whether ``features`` carries every feature of this collection (what prefetch needs)."""
        keys = set(features.keys())
        return all(f in keys for f in self._feature_names)

    def input_dist(self, features: KeyedJaggedTensor) -> dict:
        """torchrec input_dist: KJT permute to the EBC's feature order, TW keys grouped by owner, RW
        ids block-bucketized, then the counts / lengths / ids all-to-alls; returns the local KJTs."""
        if list(features.keys()) != self._feature_names:
            idx = [list(features.keys()).index(f) for f in self._feature_names]
            features = features.permute(idx)
        B = features.stride()
        values = features.values()
        if values.dtype not in (torch.int32, torch.int64):
            values = values.to(torch.int64)
        lengths = features.lengths().to(torch.int32)
        return self._input_dist_impl(values, lengths, B)

    def _input_dist_impl(self, values: torch.Tensor, lengths: torch.Tensor, B: int) -> dict:
        be, W, pg, dev = self._be, self._W, self._pg, self._device
        F = len(self._feature_names)
        offsets = be.complete_cumsum(lengths)
        idt = values.dtype
        # ---- TW: keys grouped by owner
        ntw = len(self._tw_order)
        if ntw:
            tw_l, tw_o, tw_v = be.kjt_permute(lengths, offsets, values, F, B, self._tw_order)
            bnd = [0]
            for o in range(W):
                bnd.append(bnd[-1] + len(self._tw_by_owner[o]) * B)
            tw_counts = tw_o[torch.tensor(bnd[1:], device=dev, dtype=torch.int64)] - \
                tw_o[torch.tensor(bnd[:-1], device=dev, dtype=torch.int64)]
        else:
            tw_counts = torch.zeros(W, dtype=torch.int32, device=dev)
        # ---- RW: bucketize by row block
        nrw = len(self._rw_feats)
        if nrw:
            rw_l, rw_o, rw_v = be.kjt_permute(lengths, offsets, values, F, B, self._rw_feats)
            bs = [self._rw_block[self._f_table[f]] for f in self._rw_feats]
            nl, no, nv = be.block_bucketize(rw_l, rw_o, rw_v, nrw, B, bs, W)
            idx = torch.arange(0, W + 1, device=dev, dtype=torch.int64) * (nrw * B)
            ob = no[idx]
            rw_counts = ob[1:] - ob[:-1]
        else:
            rw_counts = torch.zeros(W, dtype=torch.int32, device=dev)
        # ---- per-peer counts: [B, tw ids, rw ids]
        meta = torch.stack([torch.full((W,), B, dtype=torch.int64, device=dev), tw_counts.to(torch.int64),
                            rw_counts.to(torch.int64)], dim=1).contiguous()
        meta_recv = torch.empty_like(meta)
        dist.all_to_all_single(meta_recv, meta, group=pg)
        send = meta.cpu().tolist()
        recv = meta_recv.cpu().tolist()
        Bs = [int(x[0]) for x in recv]
        Bm = max(Bs)
        nme = len(self._tw_me)
        # ---- lengths: per peer [tw lengths for d | rw lengths for d]
        lpieces, vpieces = [], []
        for d in range(W):
            if ntw:
                a = sum(len(self._tw_by_owner[o]) for o in range(d)) * B
                lpieces.append(tw_l[a:a + len(self._tw_by_owner[d]) * B])
                va = sum(send[o][1] for o in range(d))
                vpieces.append(tw_v[va:va + send[d][1]])
            if nrw:
                lpieces.append(nl[d * nrw * B:(d + 1) * nrw * B])
                va = sum(send[o][2] for o in range(d))
                vpieces.append(nv[va:va + send[d][2]])
        l_send = torch.cat(lpieces) if lpieces else torch.zeros(0, dtype=torch.int32, device=dev)
        v_send = torch.cat(vpieces) if vpieces else torch.zeros(0, dtype=idt, device=dev)
        l_in = [(len(self._tw_by_owner[d]) + nrw) * B for d in range(W)]
        l_out = [(nme + nrw) * Bs[s] for s in range(W)]
        v_in = [send[d][1] + send[d][2] for d in range(W)]
        v_out = [recv[s][1] + recv[s][2] for s in range(W)]
        l_recv = torch.empty(sum(l_out), dtype=torch.int32, device=dev)
        v_recv = torch.empty(sum(v_out), dtype=idt, device=dev)
        _a2a(l_recv, l_send, l_out, l_in, pg)
        _a2a(v_recv, v_send, v_out, v_in, pg)
        # ---- local KJTs: keys (s, k), bag rows padded to Bm per source
        tw_lens, rw_lens, tw_vals, rw_vals = [], [], [], []
        lo = vo = 0
        for s in range(W):
            pad = Bm - Bs[s]
            blk = l_recv[lo:lo + (nme + nrw) * Bs[s]]
            lo += (nme + nrw) * Bs[s]
            tl = blk[:nme * Bs[s]].view(nme, Bs[s])
            rl = blk[nme * Bs[s]:].view(nrw, Bs[s])
            if pad:
                tl = torch.nn.functional.pad(tl, (0, pad))
                rl = torch.nn.functional.pad(rl, (0, pad))
            tw_lens.append(tl.reshape(-1))
            rw_lens.append(rl.reshape(-1))
            tw_vals.append(v_recv[vo:vo + recv[s][1]])
            vo += recv[s][1]
            rw_vals.append(v_recv[vo:vo + recv[s][2]])
            vo += recv[s][2]
        tensors = [l_recv, v_recv] + tw_lens + rw_lens + tw_vals + rw_vals
        return {"B": B, "Bm": Bm, "Bs": Bs, "tw_lens": tw_lens, "rw_lens": rw_lens, "tw_vals": tw_vals,
                "rw_vals": rw_vals, "tensors": tensors, "stream": None}

    def _lookup_output_dist(self, d: dict):
        """Local lookups on the shards, then output_dist (TW all-to-all, RW reduce-scatter)."""
        be, W, pg, dev = self._be, self._W, self._pg, self._device
        B, Bm, Bs = d["B"], d["Bm"], d["Bs"]
        tw_lens, rw_lens, tw_vals, rw_vals = d["tw_lens"], d["rw_lens"], d["tw_vals"], d["rw_vals"]
        ntw, nrw, nme = len(self._tw_order), len(self._rw_feats), len(self._tw_me)
        saved = {"B": B, "Bm": Bm, "Bs": Bs}
        out = torch.empty(B, self._out_dim, dtype=torch.float32, device=dev)
        # ---- TW lookup + output all-to-all
        if ntw:
            width_me = sum(self._dims[f] for f in self._tw_me)
            if nme:
                L = torch.cat(tw_lens)
                V = torch.cat(tw_vals)
                O = be.complete_cumsum(L)
                ts = self._lookup_ts("tw", Bm)
                pooled = torch.empty(W * Bm, width_me, dtype=torch.float32, device=dev)
                ts.pooled_fwd(V, O, Bm, pooling=self._pooling, out=pooled)
                saved["tw"] = (V, O)
            else:
                pooled = torch.empty(W * Bm, 0, dtype=torch.float32, device=dev)
            send_rows = [pooled[s * Bm:s * Bm + Bs[s]] for s in range(W)]
            p_send = torch.cat([x.reshape(-1) for x in send_rows])
            widths = [sum(self._dims[f] for f in self._tw_by_owner[o]) for o in range(W)]
            p_recv = torch.empty(sum(B * w for w in widths), dtype=torch.float32, device=dev)
            _a2a(p_recv, p_send, [B * w for w in widths], [Bs[s] * width_me for s in range(W)], pg)
            po = 0
            for o in range(W):
                if widths[o] == 0:
                    continue
                blk = p_recv[po:po + B * widths[o]].view(B, widths[o])
                po += B * widths[o]
                c = 0
                for f in self._tw_by_owner[o]:
                    out[:, self._cols[f]:self._cols[f] + self._dims[f]] = blk[:, c:c + self._dims[f]]
                    c += self._dims[f]
            saved["tw_widths"] = widths
            saved["width_me"] = width_me
        # ---- RW lookup + reduce-scatter
        if nrw:
            width_rw = sum(self._dims[f] for f in self._rw_feats)
            L = torch.cat(rw_lens)
            V = torch.cat(rw_vals)
            O = be.complete_cumsum(L)
            ts = self._lookup_ts("rw", Bm)
            partial = torch.empty(W * Bm, width_rw, dtype=torch.float32, device=dev)
            ts.pooled_fwd(V, O, Bm, pooling=self._pooling, out=partial)
            red = torch.empty(Bm, width_rw, dtype=torch.float32, device=dev)
            _reduce_scatter_rows(red, partial, W, pg)
            c = 0
            for f in self._rw_feats:
                out[:, self._cols[f]:self._cols[f] + self._dims[f]] = red[:B, c:c + self._dims[f]]
                c += self._dims[f]
            saved["rw"] = (V, O)
            saved["width_rw"] = width_rw
        return out, saved

    def _backward_impl(self, grad: torch.Tensor, saved) -> None:
        be, W, pg, dev = self._be, self._W, self._pg, self._device
        B, Bm, Bs = saved["B"], saved["Bm"], saved["Bs"]
        lr, eps = self._fused["lr"], self._fused["eps"]
        grad = grad.contiguous()
        if self._tw_order:
            widths = saved["tw_widths"]
            width_me = saved["width_me"]
            pieces = []
            for o in range(W):
                for f in self._tw_by_owner[o]:
                    pieces.append(grad[:, self._cols[f]:self._cols[f] + self._dims[f]])
            g_send = torch.cat([torch.cat([grad[:, self._cols[f]:self._cols[f] + self._dims[f]]
                                           for f in self._tw_by_owner[o]], dim=1).reshape(-1)
                                for o in range(W) if widths[o]]) if any(widths) else grad.new_zeros(0)
            g_recv = torch.empty(sum(Bs[s] * width_me for s in range(W)), dtype=torch.float32, device=dev)
            _a2a(g_recv, g_send, [Bs[s] * width_me for s in range(W)], [B * w for w in widths], pg)
            if "tw" in saved:
                g_local = torch.zeros(W * Bm, width_me, dtype=torch.float32, device=dev)
                go = 0
                for s in range(W):
                    g_local[s * Bm:s * Bm + Bs[s]] = g_recv[go:go + Bs[s] * width_me].view(Bs[s], width_me)
                    go += Bs[s] * width_me
                V, O = saved["tw"]
                ts = self._lookup_ts("tw", Bm)
                ts.bwd_prepare(V, O, Bm, max_lookups=max(1, V.numel()))
                ts.bwd_rowwise_adagrad(g_local, O, Bm, lr, eps, pooling=self._pooling)
        if self._rw_feats:
            width_rw = saved["width_rw"]
            g_rw = torch.zeros(Bm, width_rw, dtype=torch.float32, device=dev)
            c = 0
            for f in self._rw_feats:
                g_rw[:B, c:c + self._dims[f]] = grad[:, self._cols[f]:self._cols[f] + self._dims[f]]
                c += self._dims[f]
            g_all = torch.empty(W * Bm, width_rw, dtype=torch.float32, device=dev)
            _all_gather_rows(g_all, g_rw, pg)
            V, O = saved["rw"]
            ts = self._lookup_ts("rw", Bm)
            ts.bwd_prepare(V, O, Bm, max_lookups=max(1, V.numel()))
            ts.bwd_rowwise_adagrad(g_all, O, Bm, lr, eps, pooling=self._pooling)
