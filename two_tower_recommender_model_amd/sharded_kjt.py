"""The two-tower training step sharded over W MI355X for MULTI-HOT bags (BASELINE config 5: users
table-wise, items row-wise, bags of ~20 ids, B = 16,384 per rank), with fixed-size exchanges so the
whole step is captured into HIP graphs.

Semantics = DistributedModelParallel(TwoTowerTrainTask) + TrainPipelineSparseDist.progress of the
reference (03_model_training.py:798-829, :618) over TorchRec's sharded EBC: input_dist (KJT bucketized
by owner, KJTAllToAll), the owners' pooled lookups, output_dist (table-wise: all-to-all of the pooled
rows; row-wise: reduce-scatter of the partial pools), data-parallel towers (DDP mean all-reduce),
the fused row-wise Adagrad on the owners' shards over the bag gradients sent back (all-to-all /
all-gather). TorchRec's KJTAllToAll sends variable split sizes the host reads every batch
(``meta.cpu().tolist()``, torchrec/distributed/embeddingbag.py:337-339 of this repo's shim) — not
capturable. Here every exchange block has a fixed size:

  route     requester: per destination d, [lengths [F][B] of the ids d owns | those ids (row in d's
            shard), capacity ``cap``]                               (tt_kjt_route, 3 kernels)
  A         all-to-all of the id blocks                              requester -> owner
  unpack    owner: one KJT over (source s, served feature k) keys   (tt_kjt_unpack)
  prepare   owner: the backward grouping of that KJT (tt_bwd_prepare), independent of the tables
  pool      owner: tt_pooled_fwd of every (s, k) bag -> block s of exchange B, row b, column k*D
  B         all-to-all of the pooled rows (one row per (bag, owner), fp32)   owner -> requester
  sum       requester: the tower input = sum over owners (ascending) of the partial pools
            (tt_pooled_partials_sum: row-wise = TorchRec's reduce-scatter, table-wise = one term)
  T1, T2    towers fwd / bwd (bf16 MFMA) on the pooled input, weight gradients + Adam's scalars
  pack      requester: the bag gradients (dX) into the block of every owner of the feature, and the
            tower gradient x 1/W into every block               (tt_pooled_grad_pack,
                                                                 tt_tower_grads_replicated)
  C         all-to-all of the gradient blocks                        requester -> owner
  update    owner: tt_bwd_rowwise_adagrad of the grouped lookups over the received bag gradients
  Adam      every rank: the fixed-order sum of the W tower gradients (= DDP's mean all-reduce,
            identical replicas)

Every block of one exchange has ONE size (the all-to-alls use equal splits, the form captured into
graphs on this stack): exchange A's ``F*B + cap`` int32, B's ``B x Fmax*D`` fp32 (Fmax = the most
features one rank serves), C's the same plus the tower gradient's rows. ``cap`` (ids per
destination block) is sized by the caller from its resident batches (``route_counts``: max over
batches, destinations and ranks); a block over capacity or an id outside [0, N) sets sticky flags
that ``check()`` all-reduces. Lookups of one bag are pooled per owner and the owners' partials summed
in ascending owner order; the embedding gradient a row receives is the sum over ranks of the
per-rank mean-loss gradients (TorchRec's sharded EBC).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

import torch

from . import _lib, ops
from ._lib import check, id_dtype_code, ptr, stream_handle


def route_counts(values: torch.Tensor, offsets: torch.Tensor, B: int, num_embeddings: Sequence[int],
                 sharding: Sequence[str], owners: Sequence[int], W: int) -> torch.Tensor:
    """[W] ids one batch (key-major KJT, ids in range) sends to each destination (host sizing of
    ``cap``)."""
    F = len(num_embeddings)
    out = torch.zeros(W, dtype=torch.int64)
    o = offsets.cpu().to(torch.int64)
    v = values.cpu().to(torch.int64)
    for f in range(F):
        ids = v[int(o[f * B]):int(o[(f + 1) * B])]
        if sharding[f] == "row_wise":
            bs = -(-int(num_embeddings[f]) // W)
            out += torch.bincount(ids // bs, minlength=W)[:W]
        else:
            out[int(owners[f])] += ids.numel()
    return out


class FusedShardedKJTStep:
    def __init__(self, comm, num_embeddings: Sequence[int], embedding_dim: int, layer_sizes: Sequence[int],
                 batch_size: int, device: torch.device, cap: int, sharding: Optional[Sequence[str]] = None,
                 tw_owners: Optional[Sequence[int]] = None, num_query_features: int = 1, lr_emb: float = 0.01,
                 lr_dense: float = 0.01, eps: float = 1e-10, seed: int = 0,
                 full_tables: Optional[Sequence[torch.Tensor]] = None, tables: Optional[ops.TableSet] = None):
        """Features 0 .. Fq-1 feed the query tower (concatenated), Fq .. F-1 the candidate tower; one
        table per feature, ``sharding[f]`` "row_wise" (block ceil(N/W)) or "table_wise" (owner
        ``tw_owners[f]``). ``cap``: ids per destination block of exchange A. ``full_tables`` (CPU,
        optional) give the initial weights, else each rank draws its shard from U(-sqrt(1/N),
        sqrt(1/N)); tower parameters from ``seed``, identical on every rank (DDP's broadcast).
        ``tables``: adopt this rank's shards (table f = feature f's local shard; a shard of no rows
        may be a placeholder of one row, as ShardedEmbeddingBagCollection allocates) instead of
        allocating them — trained in place, not initialised (the N > 1 drop-in, dropin.py)."""
        self.comm = comm
        self.W, self.rank = comm.world, comm.rank
        W, r = self.W, self.rank
        if W > 16:
            raise _lib.TTError("sharded KJT step: at most 16 ranks")
        self.device = dev = torch.device(device)
        self.N = [int(n) for n in num_embeddings]
        self.F = F = len(self.N)
        self.Fq = int(num_query_features)
        if F < 2 or not 1 <= self.Fq < F:
            raise _lib.TTError("sharded KJT step: two towers of at least one feature each")
        self.B = B = int(batch_size)
        self.D = D = int(embedding_dim)
        if D % 32 or D > 1024:
            raise _lib.TTError("sharded KJT step: embedding dim a multiple of 32")
        self.layer_sizes = [int(x) for x in layer_sizes]
        self.lr_emb, self.lr_dense, self.eps = float(lr_emb), float(lr_dense), float(eps)
        self.sharding = list(sharding or ["row_wise"] * F)
        owners = list(tw_owners or [f % W for f in range(F)])
        self.owner = owners
        self.cap = int(cap)
        # ---- shards: one local table per feature (a dummy row where this rank holds none)
        self.block, self.row_lo, self.local_rows = [], [], []
        for f in range(F):
            if self.sharding[f] == "row_wise":
                bs = -(-self.N[f] // W)
                lo = min(r * bs, self.N[f])
                self.block.append(bs)
                self.row_lo.append(lo)
                self.local_rows.append(max(0, min(bs, self.N[f] - lo)))
            elif self.sharding[f] == "table_wise":
                self.block.append(0)
                self.row_lo.append(0)
                self.local_rows.append(self.N[f] if owners[f] == r else 0)
            else:
                raise _lib.TTError(f"sharding must be row_wise / table_wise, got {self.sharding[f]}")
        if tables is not None:
            if tables.T != F or tables.dims != [D] * F or tables.device != dev or any(
                    tables.rows[f] != self.local_rows[f] and not (self.local_rows[f] == 0 and tables.rows[f] <= 1)
                    for f in range(F)):
                raise _lib.TTError(f"sharded KJT step: adopted tables must be this rank's shards (rows "
                                   f"{self.local_rows}, dim {D}), feature f -> table f; got rows {tables.rows}")
            self.tables = tables
        else:
            self.tables = ops.TableSet([max(1, n) for n in self.local_rows], [D] * F, list(range(F)), dev)
            self.tables.weights.zero_()
        for f in range(F if tables is None else 0):
            n = self.local_rows[f]
            if not n:
                continue
            view = self.tables.table_view(f)
            if full_tables is not None:
                view[:n].copy_(full_tables[f][self.row_lo[f]:self.row_lo[f] + n])
            else:
                a = (1.0 / self.N[f]) ** 0.5
                view.uniform_(-a, a, generator=torch.Generator(device=dev).manual_seed(seed * 1000 + 17 * r + f))
        # ---- who serves what
        serves = lambda d: [f for f in range(F) if self.sharding[f] == "row_wise" or owners[f] == d]  # noqa: E731
        self.feats = serves(r)
        self.Fr = len(self.feats)
        self.Fmax = max(len(serves(d)) for d in range(W))
        col = [[-1] * F for _ in range(W)]
        for d in range(W):
            for k, f in enumerate(serves(d)):
                col[d][f] = k * D
        self._owner_col = (C.c_int32 * (W * F))(*[c for row in col for c in row])
        # ---- towers (data-parallel replicas)
        self.in_dims = [self.Fq * D, (F - self.Fq) * D]
        if not ops.FusedTowers.supported(self.in_dims, self.layer_sizes, [0, self.in_dims[0]], B):
            raise _lib.TTError("sharded KJT step: unsupported tower shape")
        self.towers = ops.FusedTowers(self.in_dims, self.layer_sizes, [0, self.in_dims[0]], B, dev)
        P = self.towers.num_params
        self.params = torch.empty(P, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(P, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(P, dtype=torch.float32, device=dev)
        self.adam_state = torch.zeros(2, dtype=torch.int64, device=dev)
        g = torch.Generator().manual_seed(seed + 1)
        chunks = []
        for t in range(2):
            i = self.in_dims[t]
            for o in self.layer_sizes:
                bound = 1.0 / i ** 0.5
                chunks += [torch.empty(o, i).uniform_(-bound, bound, generator=g).flatten(),
                           torch.empty(o).uniform_(-bound, bound, generator=g)]
                i = o
        self.params.copy_(torch.cat(chunks))
        self.towers.update(self.params, do_adam=False)
        # ---- exchange layout (identical arithmetic on every rank)
        FD = self.Fmax * D
        self.strideA = F * B + self.cap
        self.strideB = B * FD
        self.prows = -(-P // FD)
        self.strideC = (B + self.prows) * FD
        self.sendA = torch.zeros(W * self.strideA, dtype=torch.int32, device=dev)
        # receive buffers from the comm when it provides them (sharded.PeerComm: IPC-mapped for its puts)
        recv = getattr(comm, "recv_buffer", None) or (lambda shape, dtype, device: torch.zeros(shape, dtype=dtype,
                                                                                              device=device))
        self.recvA = recv((W * self.strideA,), torch.int32, dev)
        self.sendB = torch.zeros(W * self.strideB, dtype=torch.float32, device=dev)
        self.recvB = recv((W * self.strideB,), torch.float32, dev)
        self.sendC = torch.zeros(W * self.strideC, dtype=torch.float32, device=dev)
        self.recvC = recv((W * self.strideC,), torch.float32, dev)
        self.flags = torch.zeros(2, dtype=torch.int32, device=dev)  # {over capacity, id out of range}
        lib = _lib.load()
        self.route_ws = torch.empty(max(256, lib.tt_kjt_route_workspace_bytes(F, B, W)), dtype=torch.uint8, device=dev)
        Fr1 = max(1, self.Fr)
        self.unpack_ws = torch.empty(max(256, lib.tt_kjt_unpack_workspace_bytes(W, Fr1, B)), dtype=torch.uint8,
                                     device=dev)
        self.kjt_lengths = torch.zeros(W * Fr1 * B, dtype=torch.int32, device=dev)
        self.kjt_offsets = torch.zeros(W * Fr1 * B + 1, dtype=torch.int32, device=dev)
        self.kjt_values = torch.zeros(max(1, W * self.cap), dtype=torch.int32, device=dev)
        # the owner's KJT keys (s, k) -> local table feats[k]; pooled rows into block s of exchange B
        # (row s*B, column k*D), bag gradients from block s of exchange C (row s*(B + prows))
        if self.Fr:
            ft = [self.feats[k] for s in range(W) for k in range(self.Fr)]
            oo = [k * D for s in range(W) for k in range(self.Fr)]
            self.ts_fwd = self.tables.remap(ft, oo, [s * B for s in range(W) for _ in range(self.Fr)])
            self.ts_bwd = self.tables.remap(ft, oo, [s * (B + self.prows) for s in range(W) for _ in range(self.Fr)])
            self.ts_bwd.ensure_bwd_workspace(max(1, W * self.cap))
        self._ne = (C.c_int64 * F)(*self.N)
        self._bs = (C.c_int64 * F)(*self.block)
        self._ow = (C.c_int32 * F)(*owners)
        self._feats = (C.c_int32 * Fr1)(*(self.feats or [0]))
        self._tw_off = (C.c_int64 * W)(*[d * self.strideC + B * FD for d in range(W)])
        # ---- step buffers
        self.pooled = torch.zeros(B, F * D, dtype=torch.float32, device=dev)
        self.gpooled = torch.zeros(B, F * D, dtype=torch.float32, device=dev)
        self.logits = torch.empty(B, dtype=torch.float32, device=dev)
        self.loss = torch.zeros((), dtype=torch.float32, device=dev)
        self.graphs: list = []
        self._pool_inputs: list = []
        torch.cuda.synchronize(dev)

    def layer_views(self):
        """[(W, b)] per tower (query, candidate) as views of the flat parameter buffer."""
        out, o = [], 0
        for t in range(2):
            layers, i = [], self.in_dims[t]
            for n in self.layer_sizes:
                w = self.params[o:o + n * i].view(n, i)
                o += n * i
                b = self.params[o:o + n]
                o += n
                layers.append((w, b))
                i = n
            out.append(layers)
        return out

    # ---- the step ------------------------------------------------------------------------------
    def _route(self, values: torch.Tensor, offsets: torch.Tensor) -> None:
        if offsets.dtype != torch.int32 or offsets.numel() != self.F * self.B + 1:
            raise _lib.TTError("sharded KJT step: offsets must be int32 [F*B + 1]")
        check(_lib.load().tt_kjt_route(self.F, self.B, ptr(values), id_dtype_code(values.dtype), ptr(offsets),
                                       self._ne, self._bs, self._ow, self.W, self.cap, self.strideA, ptr(self.sendA),
                                       ptr(self.flags), ptr(self.route_ws), self.route_ws.numel(),
                                       stream_handle(self.device)), "kjt_route")

    def _owner_forward(self) -> None:
        """unpack -> grouping of the received lookups -> pooled rows into exchange B's blocks."""
        if not self.Fr:
            return
        W, B = self.W, self.B
        check(_lib.load().tt_kjt_unpack(W, self.F, B, ptr(self.recvA), self.strideA, self.cap, self._feats, self.Fr,
                                        ptr(self.kjt_lengths), ptr(self.kjt_offsets), ptr(self.kjt_values),
                                        ptr(self.unpack_ws), self.unpack_ws.numel(), stream_handle(self.device)),
              "kjt_unpack")
        # the backward's grouping depends on the ids only: before the pool, beside nothing
        self.ts_bwd.bwd_prepare(self.kjt_values, self.kjt_offsets, B, max_lookups=max(1, W * self.cap))
        out = self.sendB.view(W * B, self.Fmax * self.D)
        self.ts_fwd.pooled_fwd(self.kjt_values, self.kjt_offsets, B, out=out)

    def _sum_partials(self) -> None:
        check(_lib.load().tt_pooled_partials_sum(self.W, self.F, self.B, self.D, ptr(self.recvB), self.strideB,
                                                 self.Fmax * self.D, self._owner_col, ptr(self.pooled),
                                                 self.pooled.stride(0), stream_handle(self.device)),
              "pooled_partials_sum")

    def _pack_grads(self) -> None:
        lib, tw = _lib.load(), self.towers
        check(lib.tt_pooled_grad_pack(self.W, self.F, self.B, self.D, ptr(self.gpooled), self.gpooled.stride(0),
                                      self._owner_col, ptr(self.sendC), self.strideC, self.Fmax * self.D,
                                      stream_handle(self.device)), "pooled_grad_pack")
        check(lib.tt_tower_grads_replicated(C.byref(tw.shape), self.B, ptr(self.params), ptr(self.sendC), self.W,
                                            self._tw_off, 1.0 / self.W, ptr(tw.ws), tw.nbytes,
                                            stream_handle(self.device)), "tower_grads_replicated")

    def _owner_update(self) -> None:
        if not self.Fr:
            return
        g = self.recvC.view(self.W * (self.B + self.prows), self.Fmax * self.D)
        self.ts_bwd.bwd_rowwise_adagrad(g, self.kjt_offsets, self.B, self.lr_emb, self.eps)

    def _adam(self) -> None:
        tw = self.towers
        check(_lib.load().tt_tower_adam_pre_grads_sum(
            C.byref(tw.shape), self.B, ptr(self.params), self.recvC.data_ptr() + 4 * self.B * self.Fmax * self.D,
            self.W, self.strideC, ptr(self.exp_avg), ptr(self.exp_avg_sq), 1e-8, 0.9, 0.999, 0.0, ptr(tw.ws),
            tw.nbytes, None, stream_handle(self.device)), "tower_adam_pre_grads_sum")

    def step(self, values: torch.Tensor, offsets: torch.Tensor, labels: torch.Tensor) -> None:
        """One training step on this rank's KJT batch (key-major bags of F features x B, ids in range
        as the EBC takes them, complete int32 offsets) and its labels; every rank calls it with its
        own batch (collectives inside)."""
        lib, tw, comm = _lib.load(), self.towers, self.comm
        self._route(values, offsets)
        comm.all_to_all(self.recvA, self.sendA)
        self._owner_forward()
        comm.all_to_all(self.recvB, self.sendB)
        self._sum_partials()
        tw.fwd_bwd(self.pooled, self.gpooled, self.params, labels, self.logits)
        check(lib.tt_tower_wgrad_pre(C.byref(tw.shape), self.B, ptr(self.loss), ptr(tw.ws), tw.nbytes,
                                     ptr(self.adam_state), self.lr_dense, 0.9, 0.999, None, 0, 0,
                                     stream_handle(self.device)), "tower_wgrad_pre")
        self._pack_grads()
        comm.all_to_all(self.recvC, self.sendC)
        self._owner_update()
        self._adam()

    # ---- graphs over resident batches ------------------------------------------------------------
    def capture_pool(self, batches: Sequence) -> None:
        """One HIP graph per resident batch (values, offsets int32, labels int32), read in place; the
        collectives are captured (RCCL). Replay with ``run(n)`` (cyclic)."""
        if not self.comm.capturable:
            raise _lib.TTError("capture_pool: the comm is not graph-capturable")
        staged = [(v, o.to(torch.int32).contiguous(), l.to(torch.int32).contiguous()) for v, o, l in batches]
        self._pool_inputs = staged
        self._prefault_due = True  # the next replay walks the tables' pages first (TableSet.prefault)
        self.warmup()
        self.comm.retire()
        self.graphs = []
        for v, o, l in staged:
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                # thread_local: only this thread's calls are checked against the capture (the RCCL
                # watchdog's pending works are retired above, TorchComm.retire)
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    self.step(v, o, l)
            torch.cuda.current_stream(self.device).wait_stream(s)
            _lib.graph_upload(g, self.device)
            self.graphs.append(g)
        torch.cuda.synchronize(self.device)
        self.cursor = 0

    def warmup(self) -> None:
        """One eager step on a batch of empty bags (communicators, workspaces, kernels) that leaves the
        training state as it was: no id touches a table, and the towers' parameters and Adam state
        are restored."""
        keep = [t.clone() for t in (self.params, self.exp_avg, self.exp_avg_sq, self.adam_state)]
        v = torch.zeros(1, dtype=torch.int32, device=self.device)
        o = torch.zeros(self.F * self.B + 1, dtype=torch.int32, device=self.device)
        lab = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        self.step(v, o, lab)
        for t, k in zip((self.params, self.exp_avg, self.exp_avg_sq, self.adam_state), keep):
            t.copy_(k)
        self.towers.update(self.params, do_adam=False)
        torch.cuda.synchronize(self.device)

    def run(self, n: int) -> None:
        if getattr(self, "_prefault_due", False):  # first replay after a capture: the tables' pages
            self._prefault_due = False  # walked right before it (TableSet.prefault; r06pf_* profiles)
            self.tables.prefault()
        for _ in range(n):
            self.graphs[self.cursor].replay()
            self.cursor = (self.cursor + 1) % len(self.graphs)

    def run_eager(self, batches: Sequence, n: int, start: int = 0) -> None:
        for i in range(n):
            v, o, l = batches[(start + i) % len(batches)]
            self.step(v, o, l)

    def check(self, collective: bool = True) -> None:
        """Raise (on every rank) if a destination block overflowed or an id was out of range."""
        f = self.flags.clone()
        perr = getattr(self.comm, "err", None)  # PeerComm: a wait that timed out
        if perr is not None:
            f = torch.cat([f, perr])
        if collective:
            self.comm.all_reduce_max_(f)
        f = f.cpu().tolist()
        if len(f) > 2 and f[2]:
            raise _lib.TTError("sharded KJT step: a device-initiated exchange timed out waiting for a peer: results "
                               "are invalid")
        if f[0]:
            raise _lib.TTError(f"sharded KJT step: a destination block exceeded its capacity {self.cap}: results are "
                               "invalid; raise `cap`")
        if f[1]:
            raise _lib.TTError("sharded KJT step: an id outside [0, N) (the EBC takes ids in range)")

    def release_graphs(self) -> None:
        torch.cuda.synchronize(self.device)
        self.graphs = []
        self._pool_inputs = []
        import gc

        gc.collect()
        torch.cuda.synchronize(self.device)

    # ---- inspection (tests) ----------------------------------------------------------------------
    def tower_grad_sent(self) -> torch.Tensor:
        """The tower gradient x 1/W this rank sent in its last step (block 0 of exchange C)."""
        o = self.B * self.Fmax * self.D
        return self.sendC[o:o + self.towers.num_params]
