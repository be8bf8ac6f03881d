"""TEST-ONLY lookup backend for ShardedEmbeddingBagCollection on CPU tensors (gloo), built on the
oracle. The product uses ops.HIP_BACKEND; this stands in for it in the multi-process CPU tests so
the sharding / communication logic (input_dist, output_dist, their adjoints) is exercised without
a GPU. Same interface as ops.HipLookupBackend / ops.TableSet."""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from oracle import ref


class CpuTableSet:
    def __init__(self, rows, dims, feature_table, device, out_offsets=None, out_rows=None, weights=None, state=None):
        self.rows = [int(r) for r in rows]
        self.dims = [int(d) for d in dims]
        self.T = len(self.rows)
        self.feature_table = [int(t) for t in feature_table]
        self.F = len(self.feature_table)
        self.device = torch.device("cpu")
        self.tables = weights if weights is not None else [torch.empty(r, d) for r, d in zip(self.rows, self.dims)]
        self.states = state if state is not None else [torch.zeros(r) for r in self.rows]
        if out_offsets is None:
            out_offsets, o = [], 0
            for t in self.feature_table:
                out_offsets.append(o)
                o += self.dims[t]
        self.out_offsets = list(out_offsets)
        self.out_rows = list(out_rows) if out_rows is not None else [0] * self.F
        self.out_dim = max(o + self.dims[t] for o, t in zip(self.out_offsets, self.feature_table))
        self._prep = None

    def remap(self, feature_table, out_offsets, out_rows=None):
        return CpuTableSet(self.rows, self.dims, feature_table, self.device, out_offsets, out_rows, self.tables,
                           self.states)

    def table_view(self, t):
        return self.tables[t]

    def state_view(self, t):
        return self.states[t]

    def pooled_fwd(self, values, offsets, B, pooling=0, out=None):
        mode = "mean" if pooling == 1 else "sum"
        if out is None:
            out = torch.empty(max(self.out_rows) + B, self.out_dim)
        offs = offsets.to(torch.int64)
        for f, t in enumerate(self.feature_table):
            s, e = int(offs[f * B]), int(offs[(f + 1) * B])
            o = offs[f * B:(f + 1) * B + 1] - s
            pooled = torch.nn.functional.embedding_bag(values[s:e].to(torch.int64), self.tables[t], o, mode=mode,
                                                       include_last_offset=True)
            r0, c0 = self.out_rows[f], self.out_offsets[f]
            out[r0:r0 + B, c0:c0 + self.dims[t]] = pooled
        return out

    def bwd_prepare(self, values, offsets, B, max_lookups=0, bounds_check=False):
        self._prep = (values.clone(), offsets.clone(), B)

    def bwd_rowwise_adagrad(self, grad_out, offsets, B, lr, eps, pooling=0):
        values, offs, B0 = self._prep
        offs = offs.to(torch.int64)
        for t in range(self.T):
            feats = [f for f, tt in enumerate(self.feature_table) if tt == t]
            idxs, gs = [], []
            for f in feats:
                s, e = int(offs[f * B]), int(offs[(f + 1) * B])
                if e == s:
                    continue
                lens = offs[f * B + 1:(f + 1) * B + 1] - offs[f * B:(f + 1) * B]
                bag = torch.repeat_interleave(torch.arange(B), lens)
                r0, c0 = self.out_rows[f], self.out_offsets[f]
                g = grad_out[r0 + bag, c0:c0 + self.dims[t]]
                if pooling == 1:
                    g = g / lens[bag].clamp(min=1).unsqueeze(1).to(g.dtype)
                idxs.append(values[s:e].to(torch.int64))
                gs.append(g)
            if not idxs:
                continue
            idx = torch.cat(idxs)
            rows, inv = torch.unique(idx, return_inverse=True)
            grows = torch.zeros(rows.numel(), self.dims[t])
            grows.index_add_(0, inv, torch.cat(gs))
            ref.rowwise_adagrad_sparse(self.tables[t], self.states[t], rows, grows, lr, eps)


class CpuLookupBackend:
    name = "cpu-oracle"

    def table_set(self, rows, dims, feature_table, device, out_offsets=None, out_rows=None):
        return CpuTableSet(rows, dims, feature_table, device, out_offsets, out_rows)

    def complete_cumsum(self, lengths):
        return torch.from_numpy(ref.complete_cumsum(lengths.numpy()))

    def block_bucketize(self, lengths, offsets, values, F, B, block_sizes, W):
        nl, nv = ref.block_bucketize(lengths.numpy(), values.numpy(), F, B, block_sizes, W)
        nl = torch.from_numpy(nl)
        return nl, torch.from_numpy(ref.complete_cumsum(nl.numpy())), torch.from_numpy(nv).to(values.dtype)

    def kjt_permute(self, lengths, offsets, values, F, B, perm, total=None):
        l, v, _ = ref.kjt_permute(lengths.numpy(), values.numpy(), F, B, perm)
        l = torch.from_numpy(l)
        return l, torch.from_numpy(ref.complete_cumsum(l.numpy())), torch.from_numpy(v).to(values.dtype)
