"""torch-tensor wrappers over the C ABI (libtt_mi355x.so). Device tensors only; every call is
asynchronous on the current HIP stream and raises ``TTError`` on a non-zero status. There is no
CPU fallback: a CPU tensor is an error.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import (TT_BF16, TT_F32, TT_I32, TT_I64, TT_POOL_MEAN, TT_POOL_SUM, FeatureMeta, TableMeta,
                   check, id_dtype_code, ptr, ptr_array, stream_handle)


def _lib_():
    return _lib.load()


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.TTError("libtt_mi355x ops take device (HIP) tensors only; got a CPU tensor")


_WS_CACHE = {}


def scratch(nbytes: int, device: torch.device, key: str) -> torch.Tensor:
    """Per-(device, key) reusable uint8 workspace that only grows (stream-ordered reuse)."""
    k = (device.index if device.index is not None else torch.cuda.current_device(), key)
    buf = _WS_CACHE.get(k)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)
        _WS_CACHE[k] = buf
    return buf


# ---- a1/a2 ------------------------------------------------------------------------------------


def kjt_build_mod_dropzero(cols: Sequence[torch.Tensor], num_embeddings: Sequence[int],
                           values_out: Optional[torch.Tensor] = None,
                           lengths_out: Optional[torch.Tensor] = None,
                           offsets_out: Optional[torch.Tensor] = None,
                           length_per_key_out: Optional[torch.Tensor] = None):
    """Vectorised transform_to_torchrec_batch (03_model_training.py:353-371). Returns
    (values[capacity F*B], lengths[F*B] int32, offsets[F*B+1] int32, length_per_key[F] int64);
    the valid values are values[:offsets[-1]]."""
    F = len(cols)
    B = cols[0].numel()
    dev = cols[0].device
    dt = cols[0].dtype
    _dev(*cols)
    for c in cols:
        if c.dtype != dt or c.numel() != B or not c.is_contiguous():
            raise _lib.TTError("kjt_build: columns must be contiguous, same dtype and length")
    if values_out is None:
        values_out = torch.empty(F * B, dtype=dt, device=dev)
    if lengths_out is None:
        lengths_out = torch.empty(F * B, dtype=torch.int32, device=dev)
    if offsets_out is None:
        offsets_out = torch.empty(F * B + 1, dtype=torch.int32, device=dev)
    if length_per_key_out is None:
        length_per_key_out = torch.empty(F, dtype=torch.int64, device=dev)
    lib = _lib_()
    nbytes = lib.tt_kjt_build_workspace_bytes(F * B)
    ws = scratch(nbytes, dev, "kjt_build")
    colp = ptr_array(list(cols))
    ne = (C.c_int64 * F)(*[int(n) for n in num_embeddings])
    check(lib.tt_kjt_build_mod_dropzero(F, B, colp, id_dtype_code(dt), ne, ptr(values_out), ptr(lengths_out),
                                        ptr(offsets_out), ptr(length_per_key_out), ptr(ws), ws.numel(),
                                        stream_handle(dev)), "kjt_build_mod_dropzero")
    return values_out, lengths_out, offsets_out, length_per_key_out


def kjt_single_hot_cols(values: torch.Tensor, offsets: torch.Tensor, B: int, num_embeddings: Sequence[int],
                        cols_out: Sequence[torch.Tensor], err: torch.Tensor, labels: Optional[torch.Tensor] = None,
                        labels_out: Optional[torch.Tensor] = None) -> None:
    """A single-hot KJT (bags of 0 or 1 ids, key-major, complete int32 offsets [F*B+1]) -> the fused
    step's id columns (tt_kjt_single_hot_cols): 0 = empty bag, v = row v, N = row 0. ``err`` (int32 [1],
    sticky) gets bit 0 for a bag of more than one id, bit 1 for a value outside [0, N). With
    ``labels_out`` the B labels (int32 / int64) are copied to it as int32 in the same launch."""
    F = len(cols_out)
    dt = cols_out[0].dtype
    _dev(offsets, err, *cols_out)
    if offsets.dtype != torch.int32 or offsets.numel() != F * B + 1:
        raise _lib.TTError("kjt_single_hot_cols: offsets must be int32 [F*B + 1]")
    for c in cols_out:
        if c.dtype != dt or c.numel() < B or not c.is_contiguous():
            raise _lib.TTError("kjt_single_hot_cols: columns must be contiguous, one dtype, >= B ids")
    if values.numel():
        _dev(values)
        if values.dtype != dt:
            raise _lib.TTError("kjt_single_hot_cols: values must have the columns' id dtype")
        vp = ptr(values)
    else:  # every bag empty (the reference's all-zero batch gives an empty float tensor): never read
        vp = ptr(cols_out[0])
    ne = (C.c_int64 * F)(*[int(n) for n in num_embeddings])
    ldt = TT_I32
    if labels_out is not None:
        _dev(labels, labels_out)
        if labels.dtype not in (torch.int32, torch.int64) or labels.numel() < B or not labels.is_contiguous() or \
                labels_out.dtype != torch.int32 or labels_out.numel() < B:
            raise _lib.TTError("kjt_single_hot_cols: labels int32 / int64 [B] -> labels_out int32 [B]")
        ldt = id_dtype_code(labels.dtype)
    check(_lib_().tt_kjt_single_hot_cols(F, B, vp, id_dtype_code(dt), ptr(offsets), ne, ptr_array(list(cols_out)),
                                         ptr(err), ptr(labels) if labels_out is not None else None, ldt,
                                         ptr(labels_out), stream_handle(offsets.device)), "kjt_single_hot_cols")


def complete_cumsum(lengths: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _dev(lengths)
    if lengths.dtype != torch.int32:
        raise _lib.TTError("complete_cumsum: lengths must be int32")
    lengths = lengths.contiguous()
    n = lengths.numel()
    if out is None:
        out = torch.empty(n + 1, dtype=torch.int32, device=lengths.device)
    lib = _lib_()
    ws = scratch(lib.tt_complete_cumsum_workspace_bytes(n), lengths.device, "cumsum")
    check(lib.tt_complete_cumsum(ptr(lengths), n, ptr(out), ptr(ws), ws.numel(), stream_handle(lengths.device)),
          "complete_cumsum")
    return out


def kjt_permute(lengths: torch.Tensor, offsets: torch.Tensor, values: torch.Tensor, F: int, B: int,
                perm: Sequence[int], weights: Optional[torch.Tensor] = None,
                total: Optional[int] = None):
    """permute_2D_sparse_data. ``total`` = number of permuted values (computed with one device->host
    read when not given and perm is not a permutation)."""
    _dev(lengths, offsets, values, weights)
    F_out = len(perm)
    if total is None:
        if sorted(perm) == list(range(F)):
            total = values.numel()
        else:
            o = offsets.cpu()
            total = int(sum(int(o[(p + 1) * B]) - int(o[p * B]) for p in perm))
    dev = lengths.device
    out_lengths = torch.empty(F_out * B, dtype=torch.int32, device=dev)
    out_offsets = torch.empty(F_out * B + 1, dtype=torch.int32, device=dev)
    out_values = torch.empty(total, dtype=values.dtype, device=dev)
    out_weights = torch.empty(total, dtype=torch.float32, device=dev) if weights is not None else None
    p = (C.c_int32 * max(1, F_out))(*[int(x) for x in perm])
    check(_lib_().tt_kjt_permute(F, B, ptr(lengths), ptr(offsets), ptr(values), id_dtype_code(values.dtype),
                                 ptr(weights), p, F_out, ptr(out_lengths), ptr(out_offsets), ptr(out_values),
                                 ptr(out_weights), stream_handle(dev)), "kjt_permute")
    return out_lengths, out_offsets, out_values, out_weights


def block_bucketize(lengths: torch.Tensor, offsets: torch.Tensor, values: torch.Tensor, F: int, B: int,
                    block_sizes: Sequence[int], W: int, capacity: Optional[int] = None):
    """block_bucketize_sparse_features: bucket-major [W][F][B] lengths/offsets + local ids."""
    _dev(lengths, offsets, values)
    dev = lengths.device
    cap = values.numel() if capacity is None else capacity
    new_lengths = torch.empty(W * F * B, dtype=torch.int32, device=dev)
    new_offsets = torch.empty(W * F * B + 1, dtype=torch.int32, device=dev)
    new_values = torch.empty(cap, dtype=values.dtype, device=dev)
    lib = _lib_()
    ws = scratch(lib.tt_block_bucketize_workspace_bytes(F, B, W), dev, "bucketize")
    bsz = (C.c_int64 * F)(*[int(b) for b in block_sizes])
    check(lib.tt_block_bucketize(F, B, ptr(lengths), ptr(offsets), ptr(values), id_dtype_code(values.dtype), bsz, W,
                                 ptr(new_lengths), ptr(new_offsets), ptr(new_values), ptr(ws), ws.numel(),
                                 stream_handle(dev)), "block_bucketize")
    return new_lengths, new_offsets, new_values


# ---- a4 / a8: embedding tables ----------------------------------------------------------------


# TableSet buffers of at least this many bytes come from tt_table_alloc (physically contiguous when
# the driver can: -0.45 us a north-star step against the caching allocator, profiles/r06al_alloc.log)
TABLE_ALLOC_MIN_BYTES = 256 << 20


# tt_table_alloc memory whose last view is gone, freed at the next table allocation (or free_tables)
# rather than in __del__: a garbage collection can run inside a graph capture or while a stream
# still reads the buffer, and hipFree there would break the capture
_PENDING_FREE: List[Tuple[int, int]] = []


def free_tables() -> None:
    """Free the table memory no tensor refers to any more (synchronises the devices involved).
    Outside a capture only; table_empty calls it before allocating."""
    if not _PENDING_FREE or torch.cuda.is_current_stream_capturing():
        return
    for dev in sorted({d for _, d in _PENDING_FREE}):
        torch.cuda.synchronize(dev)
    while _PENDING_FREE:
        p, _ = _PENDING_FREE.pop()
        check(_lib_().tt_table_free(p), "table_free")


class _TableMemory:
    """One tt_table_alloc allocation as __cuda_array_interface__ bytes for torch.as_tensor; the
    tensor keeps this object alive, and with the last view the memory joins _PENDING_FREE."""

    def __init__(self, nbytes: int, device: torch.device):
        free_tables()
        p, flag = C.c_void_p(), C.c_int(0)
        with torch.cuda.device(device):
            check(_lib_().tt_table_alloc(nbytes, C.byref(p), C.byref(flag)), "table_alloc")
        self.ptr, self.contiguous = p.value, bool(flag.value)
        self.device = device.index if device.index is not None else torch.cuda.current_device()
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (self.ptr, False),
                                         "version": 2}

    def __del__(self):
        if self.ptr:
            _PENDING_FREE.append((self.ptr, self.device))
            self.ptr = None


def table_empty(n: int, device: torch.device, dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """An uninitialised 1-D device tensor for table storage: tt_table_alloc memory at
    TABLE_ALLOC_MIN_BYTES and above, the caching allocator below."""
    nbytes = n * torch.tensor([], dtype=dtype).element_size()
    if nbytes < TABLE_ALLOC_MIN_BYTES or torch.device(device).type != "cuda":
        return torch.empty(n, dtype=dtype, device=device)
    mem = _TableMemory(nbytes, torch.device(device))
    return torch.as_tensor(mem, device=device).view(dtype)


class TableSet:
    """Flat fp32 weight buffer + flat row-wise state for T local tables (FBGEMM-TBE-style layout:
    one allocation, per-table element offsets), with the feature->table map of a KJT.

    ``dims[t]``, ``rows[t]``: table shapes; ``feature_table[f]``: table of KJT key f;
    ``out_offsets[f]``: first column of key f in the pooled output (default: cumulative)."""

    def __init__(self, rows: Sequence[int], dims: Sequence[int], feature_table: Sequence[int],
                 device: torch.device, out_offsets: Optional[Sequence[int]] = None,
                 weights: Optional[torch.Tensor] = None, align: int = 4,
                 out_rows: Optional[Sequence[int]] = None):
        self.rows = [int(r) for r in rows]
        self.dims = [int(d) for d in dims]
        self.T = len(self.rows)
        self.feature_table = [int(t) for t in feature_table]
        self.F = len(self.feature_table)
        if not (1 <= self.T <= _lib.TT_MAX_TABLES and 1 <= self.F <= _lib.TT_MAX_FEATURES):
            raise _lib.TTError("TableSet: 1..64 tables and features supported")
        self.device = torch.device(device)
        woff, soff = [], []
        w = s = 0
        for r, d in zip(self.rows, self.dims):
            woff.append(w)
            soff.append(s)
            w += (r * d + align - 1) // align * align
            s += r
        self.weight_offsets = woff
        self.state_offsets = soff
        self.total_weights = w
        self.total_rows = s
        if weights is None:
            weights = table_empty(max(1, w), self.device)
        self.weights = weights
        self.state = table_empty(max(1, s), self.device).zero_()
        if out_offsets is None:
            out_offsets, o = [], 0
            for t in self.feature_table:
                out_offsets.append(o)
                o += self.dims[t]
        self.out_offsets = [int(o) for o in out_offsets]
        self.out_dim = max(o + self.dims[t] for o, t in zip(self.out_offsets, self.feature_table))
        self.out_rows = [int(r) for r in out_rows] if out_rows is not None else [0] * self.F
        self._tm = (TableMeta * self.T)()
        for t in range(self.T):
            self._tm[t].weight_offset = self.weight_offsets[t]
            self._tm[t].state_offset = self.state_offsets[t]
            self._tm[t].num_rows = self.rows[t]
            self._tm[t].dim = self.dims[t]
        self._fm = (FeatureMeta * self.F)()
        for f, t in enumerate(self.feature_table):
            self._fm[f].table = t
            self._fm[f].out_offset = self.out_offsets[f]
            self._fm[f].out_row = self.out_rows[f]
        self._bwd_ws = None
        self._bwd_cap = 0
        self.err_count = torch.zeros(1, dtype=torch.int32, device=self.device)

    def remap(self, feature_table: Sequence[int], out_offsets: Sequence[int],
              out_rows: Optional[Sequence[int]] = None) -> "TableSet":
        """Same tables and storage, another KJT key -> table / output-placement map."""
        ts = TableSet(self.rows, self.dims, feature_table, self.device, out_offsets=out_offsets, weights=self.weights,
                      out_rows=out_rows)
        ts.state = self.state
        return ts

    @classmethod
    def view_of(cls, src: Optional["TableSet"], table_ids: Sequence[Optional[int]], dims: Sequence[int],
                device: torch.device) -> "TableSet":
        """Tables ``table_ids[t]`` of ``src`` as tables t of a new TableSet over the SAME weight and
        state storage (feature t -> table t); ``None`` (or no ``src``): a table of 0 rows (a shard
        this rank does not hold: every key of it is out of range, so no kernel touches storage for
        it). What a step uses to train the shards a ShardedEmbeddingBagCollection already holds."""
        n = len(table_ids)
        if src is None:  # nothing held here: one zero element of storage behind every empty table
            src = cls([0], [int(dims[0])], [0], device)
        rows = [src.rows[i] if i is not None else 0 for i in table_ids]
        ts = cls(rows, [int(d) for d in dims], list(range(n)), device, weights=src.weights)
        ts.state = src.state
        for t, i in enumerate(table_ids):
            if i is not None and src.dims[i] != ts.dims[t]:
                raise _lib.TTError("TableSet.view_of: table dims differ")
            ts.weight_offsets[t] = src.weight_offsets[i] if i is not None else 0
            ts.state_offsets[t] = src.state_offsets[i] if i is not None else 0
            ts._tm[t].weight_offset = ts.weight_offsets[t]
            ts._tm[t].state_offset = ts.state_offsets[t]
        return ts

    def table_view(self, t: int) -> torch.Tensor:
        o = self.weight_offsets[t]
        return self.weights[o:o + self.rows[t] * self.dims[t]].view(self.rows[t], self.dims[t])

    def state_view(self, t: int) -> torch.Tensor:
        o = self.state_offsets[t]
        return self.state[o:o + self.rows[t]]

    def init_uniform_(self, generator: Optional[torch.Generator] = None) -> None:
        """torchrec EmbeddingBagCollection default init: U(-sqrt(1/N), sqrt(1/N)) per table."""
        for t in range(self.T):
            a = (1.0 / max(1, self.rows[t])) ** 0.5
            self.table_view(t).uniform_(-a, a, generator=generator)

    def prefault(self, page_bytes: int = 4096, passes: int = 2) -> None:
        """Walk every page of the weights and the row-wise state (tt_table_prefault, one 4-byte load
        per page, on the current stream), ``passes`` times: setup before a run's first step, so its
        first ~30 steps do not pay the cold page-table walks (profiles/r06dr_overhead4.log: +2 us a
        step over a 20-step run in a fresh process). One pass from cold took 1.4 ms and left the
        first run ~1 us a step slow; a second (0.4 ms) took off ~0.4 us more, four passes were
        worse than two (the walks' lines displace the run's own; profiles/r06pf6_overhead.log)."""
        if not hasattr(self, "_sink"):
            self._sink = torch.zeros(1, dtype=torch.int32, device=self.device)
        for buf in [self.weights, self.state] * passes:
            check(_lib_().tt_table_prefault(ptr(buf), buf.numel() * buf.element_size(), page_bytes, ptr(self._sink),
                                            stream_handle(self.device)), "table_prefault")

    # -- forward
    def pooled_fwd(self, values: torch.Tensor, offsets: torch.Tensor, B: int, pooling: int = TT_POOL_SUM,
                   out: Optional[torch.Tensor] = None, bounds_check: bool = False) -> torch.Tensor:
        _dev(values, offsets)
        if offsets.dtype != torch.int32:
            raise _lib.TTError("pooled_fwd: offsets must be int32")
        if out is None:
            out = torch.empty(max(self.out_rows) + B, self.out_dim, dtype=torch.float32, device=self.device)
        ldo = out.stride(0) if out.dim() == 2 else self.out_dim
        idt = id_dtype_code(values.dtype) if values.numel() else TT_I64
        check(_lib_().tt_pooled_fwd(ptr(self.weights), self._tm, self.T, self._fm, self.F, B, ptr(values), idt,
                                    ptr(offsets), pooling, ptr(out), ldo, 1 if bounds_check else 0,
                                    ptr(self.err_count), stream_handle(self.device)), "pooled_fwd")
        return out

    # -- backward (dedup + fused row-wise Adagrad)
    def ensure_bwd_workspace(self, max_lookups: int) -> None:
        max_lookups = max(1, int(max_lookups))
        if self._bwd_ws is not None and max_lookups <= self._bwd_cap:
            return
        cap = 1
        while cap < max_lookups:
            cap <<= 1
        lib = _lib_()
        nbytes = lib.tt_bwd_workspace_bytes(cap)
        self._bwd_ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        self._bwd_cap = cap
        check(lib.tt_bwd_workspace_init(ptr(self._bwd_ws), nbytes, cap, stream_handle(self.device)), "bwd_ws_init")

    def use_bwd_workspace(self, k: int) -> None:
        """Select grouping workspace k (0 or 1) for the following tt_bwd_prepare /
        tt_bwd_rowwise_adagrad calls: a pipelined caller groups batch i+1 into one workspace while
        batch i's update reads the other. Workspace 1 is allocated (same capacity) on first use."""
        if self._bwd_ws is None:
            raise _lib.TTError("use_bwd_workspace: call ensure_bwd_workspace first")
        if not hasattr(self, "_bwd_wss"):
            self._bwd_wss = [self._bwd_ws, None]
        if self._bwd_wss[0] is not self._bwd_ws and self._bwd_wss[1] is not self._bwd_ws:
            self._bwd_wss = [self._bwd_ws, None]  # the workspace was re-sized
        if self._bwd_wss[k] is None:
            ws = torch.empty_like(self._bwd_wss[0])
            check(_lib_().tt_bwd_workspace_init(ptr(ws), ws.numel(), self._bwd_cap, stream_handle(self.device)),
                  "bwd_ws_init")
            self._bwd_wss[k] = ws
        self._bwd_ws = self._bwd_wss[k]

    def bwd_prepare(self, values: torch.Tensor, offsets: torch.Tensor, B: int, max_lookups: int,
                    bounds_check: bool = False) -> None:
        self.ensure_bwd_workspace(max_lookups)
        idt = id_dtype_code(values.dtype) if values.numel() else TT_I64
        check(_lib_().tt_bwd_prepare(self._tm, self.T, self._fm, self.F, B, ptr(values), idt, ptr(offsets),
                                     1 if bounds_check else 0, ptr(self._bwd_ws), self._bwd_ws.numel(),
                                     self._bwd_cap, stream_handle(self.device)), "bwd_prepare")

    # -- single-hot column form (the loader's [B] id columns; transform applied inline)
    def pooled_fwd_cols(self, cols: Sequence[torch.Tensor], num_embeddings: Sequence[int],
                        out: Optional[torch.Tensor] = None) -> torch.Tensor:
        _dev(*cols)
        B = cols[0].numel()
        if out is None:
            out = torch.empty(max(self.out_rows) + B, self.out_dim, dtype=torch.float32, device=self.device)
        ne = (C.c_int64 * self.F)(*[int(n) for n in num_embeddings])
        check(_lib_().tt_pooled_fwd_cols(ptr(self.weights), self._tm, self.T, self._fm, self.F, B, ptr_array(list(cols)),
                                         id_dtype_code(cols[0].dtype), ne, ptr(out), out.stride(0),
                                         stream_handle(self.device)), "pooled_fwd_cols")
        return out

    def bwd_prepare_cols(self, cols: Sequence[torch.Tensor], num_embeddings: Sequence[int]) -> None:
        B = cols[0].numel()
        self.ensure_bwd_workspace(self.F * B)
        ne = (C.c_int64 * self.F)(*[int(n) for n in num_embeddings])
        check(_lib_().tt_bwd_prepare_cols(self._tm, self.T, self._fm, self.F, B, ptr_array(list(cols)),
                                          id_dtype_code(cols[0].dtype), ne, ptr(self._bwd_ws), self._bwd_ws.numel(),
                                          self._bwd_cap, stream_handle(self.device)), "bwd_prepare_cols")

    def bwd_rowwise_adagrad(self, grad_out: torch.Tensor, offsets: Optional[torch.Tensor], B: int, lr: float,
                            eps: float, pooling: int = TT_POOL_SUM, part: int = 0) -> None:
        """part 0: every touched row; 1: the rows looked up once (KJT form); 2: the others
        (tt_bwd_rowwise_adagrad_part: the two parts touch disjoint rows, two streams may run them)."""
        _dev(grad_out)
        if grad_out.dtype != torch.float32 or grad_out.stride(1) != 1:
            raise _lib.TTError("bwd: grad_out must be fp32 with unit column stride")
        if part:
            check(_lib_().tt_bwd_rowwise_adagrad_part(self._tm, self.T, self._fm, self.F, B, ptr(grad_out),
                                                      grad_out.stride(0), ptr(offsets), pooling, ptr(self.weights),
                                                      ptr(self.state), float(lr), float(eps), ptr(self._bwd_ws),
                                                      self._bwd_ws.numel(), self._bwd_cap, int(part),
                                                      stream_handle(self.device)), "bwd_rowwise_adagrad_part")
            return
        check(_lib_().tt_bwd_rowwise_adagrad(self._tm, self.T, self._fm, self.F, B, ptr(grad_out),
                                             grad_out.stride(0), ptr(offsets), pooling, ptr(self.weights),
                                             ptr(self.state), float(lr), float(eps), ptr(self._bwd_ws),
                                             self._bwd_ws.numel(), self._bwd_cap, stream_handle(self.device)),
              "bwd_rowwise_adagrad")

    # -- single-hot two-launch dedup + fused row-wise Adagrad (csrc/dedup.hip)
    def ensure_dedup_workspace(self, max_lookups: int) -> None:
        max_lookups = max(1, int(max_lookups))
        if getattr(self, "_dd_ws", None) is not None and max_lookups <= self._dd_cap:
            return
        lib = _lib_()
        nbytes = lib.tt_dedup_workspace_bytes(max_lookups)
        self._dd_ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        self._dd_cap = max_lookups
        check(lib.tt_dedup_workspace_init(ptr(self._dd_ws), nbytes, max_lookups, stream_handle(self.device)),
              "dedup_workspace_init")

    def dedup_insert_cols(self, cols: Sequence[torch.Tensor], num_embeddings: Sequence[int]) -> None:
        """Lookup i = f*B + b of the single-hot columns (id 0 dropped, id mod N) joins its row's slot."""
        _dev(*cols)
        B = cols[0].numel()
        self.ensure_dedup_workspace(self.F * B)
        ne = (C.c_int64 * self.F)(*[int(n) for n in num_embeddings])
        check(_lib_().tt_dedup_insert_cols(self._tm, self.T, self._fm, self.F, B, ptr_array(list(cols)),
                                           id_dtype_code(cols[0].dtype), ne, ptr(self._dd_ws), self._dd_ws.numel(),
                                           self._dd_cap, stream_handle(self.device)), "dedup_insert_cols")

    def dedup_insert_segments(self, keys: torch.Tensor, counts: torch.Tensor, seg_capacity: int) -> None:
        """Lookup i = s*C + k (k < counts[s]) with key keys[i] = table << 40 | local row."""
        _dev(keys, counts)
        if keys.dtype != torch.int64 or counts.dtype != torch.int32:
            raise _lib.TTError("dedup_insert_segments: int64 keys and int32 counts expected")
        nseg = counts.numel()
        if keys.numel() < nseg * seg_capacity:
            raise _lib.TTError("dedup_insert_segments: keys shorter than segments x capacity")
        self.ensure_dedup_workspace(nseg * seg_capacity)
        check(_lib_().tt_dedup_insert_segments(ptr(keys), ptr(counts), nseg, int(seg_capacity), ptr(self._dd_ws),
                                               self._dd_ws.numel(), self._dd_cap, stream_handle(self.device)),
              "dedup_insert_segments")

    def dedup_resolve(self) -> None:
        """Finish the dedup inserts a fused T1 (``FusedTowers.fwd_bwd_gather(dedup=...)``) deferred."""
        check(_lib_().tt_dedup_resolve(ptr(self._dd_ws), self._dd_ws.numel(), self._dd_cap,
                                       stream_handle(self.device)), "dedup_resolve")

    def dedup_rowwise_adagrad(self, grad: torch.Tensor, B: int, lr: float, eps: float, flat: bool = False) -> None:
        """Fused row-wise Adagrad over the rows inserted since the last call. Gradient row of lookup
        i: the KeyedTensor row of (feature i // B, bag i % B) — or, with ``flat``, row i of ``grad``."""
        _dev(grad)
        if grad.dtype != torch.float32 or grad.stride(-1) != 1:
            raise _lib.TTError("dedup_rowwise_adagrad: grad must be fp32 with unit column stride")
        if flat:
            fm = (FeatureMeta * 1)()
            fm[0].table, fm[0].out_offset, fm[0].out_row = 0, 0, 0
            F = 1
        else:
            fm, F = self._fm, self.F
        check(_lib_().tt_dedup_rowwise_adagrad(self._tm, self.T, fm, F, int(B), ptr(grad), grad.stride(0),
                                               ptr(self.weights), ptr(self.state), float(lr), float(eps),
                                               ptr(self._dd_ws), self._dd_ws.numel(), self._dd_cap,
                                               stream_handle(self.device)), "dedup_rowwise_adagrad")

    def _adagrad_role(self, fm, F: int, B: int, grad: torch.Tensor, lr: float, eps: float,
                      multi_only: int = 0) -> "_lib.AdagradRole":
        """The ADAGRAD role of a tt_launch plan over this set's tables and dedup workspace (the
        arguments of ``dedup_rowwise_adagrad``)."""
        if grad.dtype != torch.float32 or grad.stride(-1) != 1:
            raise _lib.TTError("dedup_rowwise_adagrad: grad must be fp32 with unit column stride")
        return _lib.AdagradRole(tables=self._tm, T=self.T, F=F, features=fm, B=int(B), grad=ptr(grad),
                                ldg=grad.stride(0), weights=ptr(self.weights), state=ptr(self.state), lr=float(lr),
                                eps=float(eps), dedup_ws=ptr(self._dd_ws), dedup_ws_bytes=self._dd_ws.numel(),
                                dedup_max_lookups=self._dd_cap, multi_only=multi_only)

    def bwd_dense(self, grad_out: torch.Tensor, values: torch.Tensor, offsets: torch.Tensor, B: int,
                  grad_weights: torch.Tensor, pooling: int = TT_POOL_SUM) -> None:
        _dev(grad_out, grad_weights)
        idt = id_dtype_code(values.dtype) if values.numel() else TT_I64
        check(_lib_().tt_pooled_bwd_dense(self._tm, self.T, self._fm, self.F, B, ptr(grad_out), grad_out.stride(0),
                                          ptr(values), idt, ptr(offsets), pooling, ptr(grad_weights), 0,
                                          stream_handle(self.device)), "pooled_bwd_dense")


# ---- a6: tower GEMMs --------------------------------------------------------------------------


def _x_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return TT_F32
    if t.dtype == torch.bfloat16:
        return TT_BF16
    raise _lib.TTError("linear: X must be fp32 or bf16")


def _compute_code(precision: str) -> int:
    if precision == "bf16":
        return TT_BF16
    if precision == "fp32":
        return TT_F32
    raise _lib.TTError("precision must be 'bf16' or 'fp32'")


def linear_fwd(xs: Sequence[torch.Tensor], ws: Sequence[torch.Tensor], bs: Sequence[Optional[torch.Tensor]],
               relu: bool = True, outs: Optional[Sequence[torch.Tensor]] = None,
               precision: str = "bf16") -> List[torch.Tensor]:
    """Grouped Y_g = act(X_g W_g^T + b_g) on bf16 MFMA (fp32 accumulate); X row stride may be > K
    (column slices of a KeyedTensor are consumed in place)."""
    G = len(xs)
    M, K = xs[0].shape
    N = ws[0].shape[0]
    dev = xs[0].device
    _dev(*xs, *ws)
    for x, w in zip(xs, ws):
        if x.shape != (M, K) or x.stride(1) != 1 or w.shape != (N, K) or not w.is_contiguous():
            raise _lib.TTError("linear_fwd: shape/stride mismatch")
    if outs is None:
        outs = [torch.empty(M, N, dtype=torch.float32, device=dev) for _ in range(G)]
    check(_lib_().tt_linear_fwd(G, ptr_array(xs), _x_code(xs[0]), xs[0].stride(0), ptr_array(ws), ptr_array(bs),
                                M, N, K, ptr_array(outs), outs[0].stride(0), 1 if relu else 0,
                                _compute_code(precision), stream_handle(dev)), "linear_fwd")
    return list(outs)


def linear_bwd_data(dys: Sequence[torch.Tensor], ys: Sequence[Optional[torch.Tensor]], ws: Sequence[torch.Tensor],
                    relu: bool = True, outs: Optional[Sequence[torch.Tensor]] = None,
                    precision: str = "bf16") -> List[torch.Tensor]:
    G = len(dys)
    M, N = dys[0].shape
    K = ws[0].shape[1]
    dev = dys[0].device
    _dev(*dys, *ws)
    if outs is None:
        outs = [torch.empty(M, K, dtype=torch.float32, device=dev) for _ in range(G)]
    check(_lib_().tt_linear_bwd_data(G, ptr_array(dys), ptr_array(ys if relu else [None] * G), dys[0].stride(0),
                                     ptr_array(ws), M, N, K, ptr_array(outs), outs[0].stride(0), 1 if relu else 0,
                                     _compute_code(precision), stream_handle(dev)), "linear_bwd_data")
    return list(outs)


def linear_bwd_weight(dys: Sequence[torch.Tensor], ys: Sequence[Optional[torch.Tensor]], xs: Sequence[torch.Tensor],
                      relu: bool = True, dws: Optional[Sequence[torch.Tensor]] = None,
                      dbs: Optional[Sequence[Optional[torch.Tensor]]] = None, precision: str = "bf16"):
    G = len(dys)
    M, N = dys[0].shape
    K = xs[0].shape[1]
    dev = dys[0].device
    _dev(*dys, *xs)
    if dws is None:
        dws = [torch.empty(N, K, dtype=torch.float32, device=dev) for _ in range(G)]
    if dbs is None:
        dbs = [torch.empty(N, dtype=torch.float32, device=dev) for _ in range(G)]
    lib = _lib_()
    ws = scratch(lib.tt_linear_bwd_weight_workspace_bytes(G, M, N, K), dev, "bwd_weight")
    check(lib.tt_linear_bwd_weight(G, ptr_array(dys), ptr_array(ys if relu else [None] * G), dys[0].stride(0),
                                   ptr_array(xs), _x_code(xs[0]), xs[0].stride(0), M, N, K, ptr_array(dws),
                                   ptr_array(dbs), 1 if relu else 0, _compute_code(precision), ptr(ws), ws.numel(),
                                   stream_handle(dev)),
          "linear_bwd_weight")
    return list(dws), list(dbs)


# ---- a7 / a9 ----------------------------------------------------------------------------------


class DotBCE:
    """logits = (q*c).sum(1); loss = BCEWithLogits mean; optional dq, dc (k5). Owns its workspace."""

    def __init__(self, device: torch.device, max_batch: int):
        self.device = torch.device(device)
        self.max_batch = int(max_batch)
        lib = _lib_()
        self.nbytes = lib.tt_dot_bce_workspace_bytes(self.max_batch)
        self.ws = torch.empty(self.nbytes, dtype=torch.uint8, device=self.device)
        check(lib.tt_dot_bce_workspace_init(ptr(self.ws), self.nbytes, self.max_batch, stream_handle(self.device)),
              "dot_bce_ws_init")

    def __call__(self, q, c, labels, logits=None, loss=None, dq=None, dc=None, grad_scale: float = 1.0):
        B, dim = q.shape
        if B > self.max_batch:
            raise _lib.TTError("DotBCE: batch exceeds workspace")
        _dev(q, c, labels)
        if logits is None:
            logits = torch.empty(B, dtype=torch.float32, device=q.device)
        if loss is None:
            loss = torch.empty((), dtype=torch.float32, device=q.device)
        ldt = {torch.int32: TT_I32, torch.int64: TT_I64, torch.float32: TT_F32}.get(labels.dtype)
        if ldt is None:
            raise _lib.TTError("DotBCE: labels must be int32/int64/float32")
        check(_lib_().tt_dot_bce_fwd_bwd(ptr(q), q.stride(0), ptr(c), c.stride(0), B, dim, ptr(labels), ldt,
                                         ptr(logits), ptr(loss), ptr(dq), dq.stride(0) if dq is not None else 0,
                                         ptr(dc), dc.stride(0) if dc is not None else 0, float(grad_scale),
                                         ptr(self.ws), self.nbytes, stream_handle(q.device)), "dot_bce")
        return logits, loss


def adam_step(params: torch.Tensor, grads: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor,
              step_state: torch.Tensor, lr: float, beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8,
              weight_decay: float = 0.0) -> None:
    _dev(params, grads, exp_avg, exp_avg_sq, step_state)
    check(_lib_().tt_adam_step(ptr(params), ptr(grads), ptr(exp_avg), ptr(exp_avg_sq), params.numel(), float(lr),
                               float(beta1), float(beta2), float(eps), float(weight_decay), ptr(step_state),
                               stream_handle(params.device)), "adam_step")


class HipLookupBackend:
    """The compute backend of the sharded lookup (ShardedEmbeddingBagCollection): table storage,
    pooled forward, fused backward and the KJT integer ops, all on libtt_mi355x.so."""

    name = "hip"

    def table_set(self, rows, dims, feature_table, device, out_offsets=None, out_rows=None) -> TableSet:
        return TableSet(rows, dims, feature_table, device, out_offsets=out_offsets, out_rows=out_rows)

    def complete_cumsum(self, lengths: torch.Tensor) -> torch.Tensor:
        return complete_cumsum(lengths)

    def block_bucketize(self, lengths, offsets, values, F, B, block_sizes, W):
        return block_bucketize(lengths, offsets, values, F, B, block_sizes, W)

    def kjt_permute(self, lengths, offsets, values, F, B, perm, total=None):
        l, o, v, _ = kjt_permute(lengths, offsets, values, F, B, perm, total=total)
        return l, o, v


HIP_BACKEND = HipLookupBackend()


# ---- a6 + a7 + a9 fused: the towers' step in three launches -----------------------------------


class FusedTowers:
    """Both towers (L layers of Linear + ReLU), dot + BCE and Adam as three kernels (T1 fwd/bwd,
    T2 weight gradients, T3 reduce + Adam + bf16 weight copies). Parameter layout: see
    tt_tower_shape_t in include/tt_mi355x.h. bf16 operands, fp32 accumulation."""

    @staticmethod
    def supported(in_dims: Sequence[int], widths: Sequence[int], in_cols: Sequence[int], B: int) -> bool:
        return (1 <= len(widths) <= 4 and all(w % 32 == 0 and 32 <= w <= 128 for w in widths)
                and all(d % 32 == 0 and 32 <= d <= 1024 for d in in_dims) and all(c % 4 == 0 for c in in_cols)
                and B % 8 == 0 and B >= 8)

    def __init__(self, in_dims: Sequence[int], widths: Sequence[int], in_cols: Sequence[int], B: int,
                 device: torch.device, flags: int = 0):
        """flags: _lib.TT_TOWER_GENERAL_T1 when T1 always runs the general kernel (several features
        per tower)."""
        self.device = torch.device(device)
        self.B = int(B)
        sh = _lib.TowerShape()
        sh.flags = int(flags)
        sh.L = len(widths)
        for i, w in enumerate(widths):
            sh.width[i] = int(w)
        for t in range(2):
            sh.in_dim[t] = int(in_dims[t])
            sh.in_col[t] = int(in_cols[t])
        self.shape = sh
        lib = _lib_()
        self.num_params = lib.tt_tower_num_params(C.byref(sh))
        if self.num_params < 0:
            check(1001, "tower shape")
        self.nbytes = lib.tt_tower_workspace_bytes(C.byref(sh), self.B)
        if self.nbytes == 0:
            check(1001, "tower shape")
        self.ws = torch.empty(self.nbytes, dtype=torch.uint8, device=self.device)
        check(lib.tt_tower_workspace_init(C.byref(sh), self.B, ptr(self.ws), self.nbytes,
                                          stream_handle(self.device)), "tower_workspace_init")

    def fwd_bwd(self, pooled, gpooled, params, labels, logits, grad_scale: float = 1.0) -> None:
        """T1. The scalar loss of this pass is written by the following wgrad()."""
        ldt = {torch.int32: TT_I32, torch.int64: TT_I64, torch.float32: TT_F32}[labels.dtype]
        if pooled.stride(0) != gpooled.stride(0):
            raise ValueError("pooled and its gradient must share a row stride")
        check(_lib_().tt_tower_fwd_bwd(C.byref(self.shape), self.B, ptr(pooled), pooled.stride(0), ptr(gpooled),
                                       ptr(params), ptr(labels), ldt, float(grad_scale), ptr(logits),
                                       ptr(self.ws), self.nbytes, stream_handle(self.device)), "tower_fwd_bwd")

    def fwd_bwd_gather(self, cols, num_embeddings, table_rows, gpooled, params, labels, logits,
                       pooled_out=None, grad_scale: float = 1.0, dedup: Optional["TableSet"] = None,
                       dedup_tables: Sequence[int] = (0, 1)) -> None:
        """T1 with the single-hot EBC forward fused in: tower t's input rows are gathered from the
        table view ``table_rows[t]`` ([rows, in_dim[t]] fp32) by ``cols[t] % num_embeddings[t]``
        (id 0 -> zeros). ``pooled_out`` (optional) receives the gathered rows. With ``dedup`` (the
        TableSet whose dedup workspace the next ``dedup_rowwise_adagrad`` reads) the lookups are
        also inserted (tower t -> table ``dedup_tables[t]``)."""
        ldt = {torch.int32: TT_I32, torch.int64: TT_I64, torch.float32: TT_F32}[labels.dtype]
        for t in range(2):
            if table_rows[t].shape[1] != self.shape.in_dim[t] or int(num_embeddings[t]) > table_rows[t].shape[0]:
                raise _lib.TTError("fwd_bwd_gather: table view does not match the tower input")
        if pooled_out is not None and pooled_out.stride(0) != gpooled.stride(0):
            raise ValueError("pooled_out and the gradient must share a row stride")
        ne = (C.c_int64 * 2)(*[int(n) for n in num_embeddings])
        dd_tab, dd_ws, dd_bytes, dd_cap = None, None, 0, 0
        if dedup is not None:
            dedup.ensure_dedup_workspace(2 * self.B)
            dd_tab = (C.c_int32 * 2)(*[int(t) for t in dedup_tables])
            dd_ws, dd_bytes, dd_cap = dedup._dd_ws, dedup._dd_ws.numel(), dedup._dd_cap
        check(_lib_().tt_tower_fwd_bwd_gather(C.byref(self.shape), self.B, ptr_array(list(cols)),
                                              id_dtype_code(cols[0].dtype), ne, ptr_array(list(table_rows)),
                                              ptr(pooled_out), gpooled.stride(0), ptr(gpooled), ptr(params),
                                              ptr(labels), ldt, float(grad_scale), ptr(logits), dd_tab, ptr(dd_ws),
                                              dd_bytes, dd_cap, ptr(self.ws), self.nbytes,
                                              stream_handle(self.device)), "tower_fwd_bwd_gather")

    def fwd_bwd_kjt(self, values, offsets, table_rows, gpooled, params, labels, logits, pooled_out=None,
                    grad_scale: float = 1.0) -> None:
        """T1 with the multi-hot EBC forward fused in: tower t's input row m is the sum pool of bag
        (t, m) of the key-major KJT (``values``, complete int32 ``offsets`` [2B + 1]) over the table
        view ``table_rows[t]`` ([rows, in_dim[t]] fp32); bit-identical to ``pooled_fwd`` + ``fwd_bwd``.
        ``pooled_out`` (optional) receives the pooled rows."""
        ldt = {torch.int32: TT_I32, torch.int64: TT_I64, torch.float32: TT_F32}[labels.dtype]
        if offsets.dtype != torch.int32 or offsets.numel() != 2 * self.B + 1:
            raise _lib.TTError("fwd_bwd_kjt: offsets must be int32 [2B + 1]")
        for t in range(2):
            if table_rows[t].shape[1] != self.shape.in_dim[t] or not table_rows[t].is_contiguous():
                raise _lib.TTError("fwd_bwd_kjt: table view does not match the tower input")
        if pooled_out is not None and pooled_out.stride(0) != gpooled.stride(0):
            raise ValueError("pooled_out and the gradient must share a row stride")
        nr = (C.c_int64 * 2)(*[int(table_rows[t].shape[0]) for t in range(2)])
        check(_lib_().tt_tower_fwd_bwd_kjt(C.byref(self.shape), self.B, ptr(values), id_dtype_code(values.dtype),
                                           ptr(offsets), nr, ptr_array(list(table_rows)), ptr(pooled_out),
                                           gpooled.stride(0), ptr(gpooled), ptr(params), ptr(labels), ldt,
                                           float(grad_scale), ptr(logits), ptr(self.ws), self.nbytes,
                                           stream_handle(self.device)), "tower_fwd_bwd_kjt")

    def fwd_bwd_indexed(self, pos, rows_in, grad_rows_out, params, labels, logits, grad_scale: float = 1.0) -> None:
        """T1 of the sharded step: tower t's input row m is ``rows_in[t][pos[t][m]]`` (-1: zeros) and
        its input gradient goes to ``grad_rows_out[t][pos[t][m]]``."""
        ldt = {torch.int32: TT_I32, torch.int64: TT_I64, torch.float32: TT_F32}[labels.dtype]
        bf16 = rows_in[0].dtype == torch.bfloat16  # rows from tt_shard_gather_rows_bf16
        for t in range(2):
            if pos[t].dtype != torch.int32 or pos[t].numel() < self.B:
                raise _lib.TTError("fwd_bwd_indexed: pos must be int32 [B]")
            for x, want in ((rows_in[t], torch.bfloat16 if bf16 else torch.float32), (grad_rows_out[t], torch.float32)):
                if x.dtype != want or x.dim() != 2 or x.shape[1] != self.shape.in_dim[t] or not x.is_contiguous():
                    raise _lib.TTError("fwd_bwd_indexed: row buffers must be contiguous [*, in_dim] (rows fp32 or "
                                       "bf16, gradient rows fp32)")
        fn = _lib_().tt_tower_fwd_bwd_indexed_bf16 if bf16 else _lib_().tt_tower_fwd_bwd_indexed
        check(fn(C.byref(self.shape), self.B, ptr_array(list(pos)),
                                               ptr_array(list(rows_in)), ptr_array(list(grad_rows_out)), ptr(params),
                                               ptr(labels), ldt, float(grad_scale), ptr(logits), ptr(self.ws),
                                               self.nbytes, stream_handle(self.device)), "tower_fwd_bwd_indexed")

    def wgrad(self, loss=None) -> None:
        """T2; also reduces T1's loss partials into loss[0] when given."""
        check(_lib_().tt_tower_wgrad(C.byref(self.shape), self.B, ptr(loss), ptr(self.ws), self.nbytes,
                                     stream_handle(self.device)), "tower_wgrad")

    def wgrad_rowwise_adagrad(self, loss, tables: "TableSet", grad: torch.Tensor, emb_B: int, lr: float, eps: float,
                              flat: bool = False, adam_step_state=None, adam_lr: float = 0.01, adam_beta1: float = 0.9,
                              adam_beta2: float = 0.999) -> None:
        """T2 and ``tables.dedup_rowwise_adagrad(grad, emb_B, lr, eps, flat)`` in one launch; with
        ``adam_step_state`` it also advances the Adam step for a following ``update_pre``."""
        _dev(grad)
        if flat:
            fm = (FeatureMeta * 1)()
            fm[0].table, fm[0].out_offset, fm[0].out_row = 0, 0, 0
            F = 1
        else:
            fm, F = tables._fm, tables.F
        _lib.launch(_lib.LaunchPlan(
            roles=_lib.ROLE_WGRAD | _lib.ROLE_ADAGRAD, shape=C.pointer(self.shape), B=self.B, workspace=ptr(self.ws),
            ws_bytes=self.nbytes,
            wgrad=_lib.WgradRole(loss=ptr(loss), adam_step_state=ptr(adam_step_state), adam_lr=float(adam_lr),
                                 adam_beta1=float(adam_beta1), adam_beta2=float(adam_beta2)),
            adagrad=tables._adagrad_role(fm, F, emb_B, grad, lr, eps)), stream_handle(self.device),
            "tower_wgrad_rowwise_adagrad")

    def wgrad_pre(self, loss, adam_step_state, adam_lr: float = 0.01, adam_beta1: float = 0.9,
                  adam_beta2: float = 0.999, dedup: Optional["TableSet"] = None) -> None:
        """T2 alone; also advances the Adam step and precomputes its scalars for ``update_pre`` /
        ``update_pre_rowwise_adagrad``. With ``dedup`` (the TableSet whose dedup workspace T1 filled)
        the same launch finishes T1's deferred inserts."""
        dws, dnb, dcap = (None, 0, 0) if dedup is None else (dedup._dd_ws, dedup._dd_ws.numel(), dedup._dd_cap)
        check(_lib_().tt_tower_wgrad_pre(C.byref(self.shape), self.B, ptr(loss), ptr(self.ws), self.nbytes,
                                         ptr(adam_step_state), float(adam_lr), float(adam_beta1), float(adam_beta2),
                                         ptr(dws), dnb, dcap, stream_handle(self.device)), "tower_wgrad_pre")

    def update_pre_rowwise_adagrad(self, params, exp_avg, exp_avg_sq, tables: "TableSet", grad: torch.Tensor,
                                   emb_B: int, lr: float, emb_eps: float, flat: bool = False, beta1: float = 0.9,
                                   beta2: float = 0.999, eps: float = 1e-8, weight_decay: float = 0.0,
                                   grads_out=None) -> None:
        """``update_pre`` and ``tables.dedup_rowwise_adagrad(grad, emb_B, lr, emb_eps, flat)`` in one launch
        (after ``wgrad_pre``)."""
        _dev(grad)
        if flat:
            fm = (FeatureMeta * 1)()
            fm[0].table, fm[0].out_offset, fm[0].out_row = 0, 0, 0
            F = 1
        else:
            fm, F = tables._fm, tables.F
        _lib.launch(_lib.LaunchPlan(
            roles=_lib.ROLE_UPDATE | _lib.ROLE_ADAGRAD, shape=C.pointer(self.shape), B=self.B, workspace=ptr(self.ws),
            ws_bytes=self.nbytes,
            update=_lib.UpdateRole(params=ptr(params), exp_avg=ptr(exp_avg), exp_avg_sq=ptr(exp_avg_sq), eps=float(eps),
                                   beta1=float(beta1), beta2=float(beta2), weight_decay=float(weight_decay),
                                   grads_out=ptr(grads_out)),
            adagrad=tables._adagrad_role(fm, F, emb_B, grad, lr, emb_eps)), stream_handle(self.device),
            "tower_update_pre_rowwise_adagrad")

    def update_pre(self, params, exp_avg, exp_avg_sq, beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8,
                   weight_decay: float = 0.0, grads_out=None) -> None:
        """T3 with the Adam scalars the preceding wgrad_rowwise_adagrad(adam_step_state=...) computed."""
        check(_lib_().tt_tower_update_pre(C.byref(self.shape), self.B, ptr(params), ptr(exp_avg), ptr(exp_avg_sq),
                                          float(eps), float(beta1), float(beta2), float(weight_decay),
                                          ptr(grads_out), ptr(self.ws), self.nbytes, stream_handle(self.device)),
              "tower_update_pre")

    def adam_grads(self, params, grads, exp_avg, exp_avg_sq, step_state, lr: float = 0.01, beta1: float = 0.9,
                   beta2: float = 0.999, eps: float = 1e-8, weight_decay: float = 0.0) -> None:
        """T3 from an explicit gradient (the all-reduced one of the data-parallel towers)."""
        check(_lib_().tt_tower_adam_grads(C.byref(self.shape), self.B, ptr(params), ptr(grads), ptr(exp_avg),
                                          ptr(exp_avg_sq), float(lr), float(beta1), float(beta2), float(eps),
                                          float(weight_decay), ptr(step_state), ptr(self.ws), self.nbytes,
                                          stream_handle(self.device)), "tower_adam_grads")

    def update(self, params, exp_avg=None, exp_avg_sq=None, step_state=None, lr: float = 0.01, beta1: float = 0.9,
               beta2: float = 0.999, eps: float = 1e-8, weight_decay: float = 0.0, do_adam: bool = True,
               grads_out=None) -> None:
        check(_lib_().tt_tower_update(C.byref(self.shape), self.B, ptr(params), ptr(exp_avg), ptr(exp_avg_sq),
                                      float(lr), float(beta1), float(beta2), float(eps), float(weight_decay),
                                      ptr(step_state), 1 if do_adam else 0, ptr(grads_out), ptr(self.ws),
                                      self.nbytes, stream_handle(self.device)), "tower_update")
