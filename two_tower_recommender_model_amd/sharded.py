"""The two-tower training step sharded over W MI355X (one process per GPU), single-hot features.

Semantics = DistributedModelParallel(TwoTowerTrainTask) + TrainPipelineSparseDist.progress of the
reference (03_model_training.py:798-829, :618): every table row-wise (block ceil(N/W)) or
table-wise sharded over the ranks, the towers data-parallel (DDP: gradients averaged over ranks),
each rank training on its own local batch of B pairs. Per step and rank:

  route           ids -> owners: segment (owner d, feature f) of fixed capacity C, pos[f][b]
                  (tt_shard_route_cols; transform_to_torchrec_batch's id % N and drop-0 inline)
  all-to-all      ids out                                   [W][F + F*C] int64
  gather          owner copies the requested rows, files each slot in its dedup table
  all-to-all      rows back                                 [W*F*C][D] fp32
  T1 (indexed)    towers fwd/bwd reading rows_in[pos], dX -> grad_out[pos]
  all-to-all      gradient rows to the owners               [W*F*C][D] fp32
  T2, T3a         towers' weight gradients, reduced (beside the gradient all-to-all)
  all-reduce      tower gradient mean over ranks (beside the owner's row-wise Adagrad)
  Adagrad         owner's fused row-wise Adagrad over the received gradient rows
  T3b             Adam from the all-reduced gradient

Every exchange has a fixed size, so with RCCL (backend "nccl") the step is captured into HIP graphs
like the single-GPU step. The embedding gradient a row receives is the sum over ranks of the
per-rank mean-loss gradients (TorchRec's sharded EBC semantics); lookups of a row are summed in
ascending (source rank, bag) order. A segment over capacity or a key outside a shard raises on
``check()`` (sticky device flags).
"""
from __future__ import annotations

import ctypes as C
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import _lib, ops
from ._lib import check, id_dtype_code, ptr, ptr_array, stream_handle


# ---- collectives --------------------------------------------------------------------------------


class _Done:
    def wait(self):
        return None


def graph_safe_nccl_env() -> None:
    """Environment for a "nccl" (RCCL) process group whose collectives are captured into HIP graphs;
    call BEFORE dist.init_process_group. ProcessGroupNCCL's watchdog queries the end events of the
    works it tracks; with its event cache on, an event of an eager collective can come back recorded
    in a capturing stream, and the query then fails (hipErrorCapturedEvent), which the watchdog
    turned into an abort of the process (seen on MI355X after a run of the graphed sharded step).
    The cache is turned off, and such a query error is logged instead of rethrown."""
    import os

    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    os.environ.setdefault("TORCH_NCCL_RETHROW_CUDA_ERRORS", "0")


class TorchComm:
    """torch.distributed collectives on the current stream (backend "nccl" = RCCL over xGMI)."""

    capturable = True

    def __init__(self, group=None, always_collective: bool = False):
        """always_collective: issue the collectives even at world size 1 (exercises RCCL, and its
        graph capture, on a one-GPU box)."""
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.always = bool(always_collective)

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        """Equal-split all-to-all along dim 0. async_op: returns a handle whose wait() makes the
        current stream wait for the collective (RCCL runs on its own stream meanwhile)."""
        if self.world == 1 and not self.always:
            out.copy_(inp)
            return _Done()
        w = dist.all_to_all_single(out, inp, group=self.group, async_op=async_op)
        return w if async_op else _Done()

    def gather_rows(self, local: torch.Tensor, spans: Sequence[Tuple[int, int]], full_rows: int):
        """Rank 0 receives every rank's row block (spans[r] = (first row, rows)) into one
        [full_rows, D] tensor (returned on rank 0, None elsewhere); point-to-point, so no rank
        ever holds more than its own shard plus, on rank 0, the result."""
        D = local.shape[1]
        if self.rank == 0:
            full = torch.empty(full_rows, D, dtype=local.dtype, device=local.device)
            lo, n = spans[0]
            full[lo:lo + n].copy_(local[:n])
            for r in range(1, self.world):
                lo, n = spans[r]
                if n:
                    buf = torch.empty(n, D, dtype=local.dtype, device=local.device)
                    dist.recv(buf, src=r, group=self.group)
                    full[lo:lo + n].copy_(buf)
            return full
        lo, n = spans[self.rank]
        if n:
            dist.send(local[:n].contiguous(), dst=0, group=self.group)
        return None

    def all_reduce_mean(self, t: torch.Tensor, async_op: bool = False):
        if self.world == 1 and not self.always:
            return _Done()
        t.mul_(1.0 / self.world)  # DDP divides by the world size, then sums
        w = dist.all_reduce(t, group=self.group, async_op=async_op)
        return w if async_op else _Done()


class ThreadComm:
    """W ranks as W threads of ONE process on one device (tests): each collective is a rendezvous
    on a barrier; all-to-all copies the peers' blocks, all-reduce sums in rank order."""

    capturable = False

    class _Shared:
        def __init__(self, world):
            self.world = world
            self.barrier = threading.Barrier(world)
            self.slots = [None] * world

    def __init__(self, shared: "ThreadComm._Shared", rank: int):
        self.shared = shared
        self.world = shared.world
        self.rank = rank

    @classmethod
    def group(cls, world: int) -> List["ThreadComm"]:
        sh = cls._Shared(world)
        return [cls(sh, r) for r in range(world)]

    def _exchange(self, t):
        torch.cuda.current_stream().synchronize()
        self.shared.slots[self.rank] = t
        self.shared.barrier.wait()

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        self._exchange(inp)
        n = out.shape[0] // self.world
        for s in range(self.world):
            src = self.shared.slots[s]
            out[s * n:(s + 1) * n].copy_(src[self.rank * n:(self.rank + 1) * n])
        torch.cuda.current_stream().synchronize()
        self.shared.barrier.wait()
        return _Done()

    def gather_rows(self, local: torch.Tensor, spans: Sequence[Tuple[int, int]], full_rows: int):
        self._exchange(local)
        full = None
        if self.rank == 0:
            full = torch.empty(full_rows, local.shape[1], dtype=local.dtype, device=local.device)
            for r in range(self.world):
                lo, n = spans[r]
                full[lo:lo + n].copy_(self.shared.slots[r][:n])
        torch.cuda.current_stream().synchronize()
        self.shared.barrier.wait()
        return full

    def all_reduce_mean(self, t: torch.Tensor, async_op: bool = False):
        self._exchange(t.clone())
        acc = None
        for s in range(self.world):
            x = self.shared.slots[s] * (1.0 / self.world)
            acc = x if acc is None else acc + x
        torch.cuda.current_stream().synchronize()
        self.shared.barrier.wait()
        t.copy_(acc)
        torch.cuda.current_stream().synchronize()
        return _Done()


# ---- the step -----------------------------------------------------------------------------------


def default_capacity(B: int, W: int, factor: float = 1.25) -> int:
    """Per-(owner, feature) segment capacity: the expected B/W lookups per owner with slack for
    the binomial spread of uniformly spread ids (B/W + 6 sigma at B = 8192, W = 8 is ~1200)."""
    if W == 1:
        return B
    c = int(factor * B / W) + 64
    return min(B, (c + 7) // 8 * 8)


class FusedShardedTwoTowerStep:
    def __init__(self, comm, num_embeddings: Sequence[int], embedding_dim: int, layer_sizes: Sequence[int],
                 batch_size: int, device: torch.device, sharding: Optional[Sequence[str]] = None,
                 tw_owners: Optional[Sequence[int]] = None, lr_emb: float = 0.01, lr_dense: float = 0.01,
                 eps: float = 1e-10, id_dtype: torch.dtype = torch.int64, seed: int = 0,
                 capacity: Optional[int] = None, full_tables: Optional[Sequence[torch.Tensor]] = None,
                 overlap_comm: bool = False):
        """Two features (query, candidate), one table each, single-hot. ``sharding[f]`` is
        "row_wise" (default) or "table_wise" (owner ``tw_owners[f]``). ``full_tables`` (CPU,
        optional) give the initial weights; otherwise each rank draws its shard from
        U(-sqrt(1/N), sqrt(1/N)) (torchrec EBC init). Tower parameters are initialised from
        ``seed`` identically on every rank (what DDP's initial broadcast guarantees).
        ``overlap_comm``: run the gradient all-to-all beside T2 and the tower all-reduce beside the
        owner's Adagrad on RCCL's stream; off by default, since each cross-stream join inside the
        step graph costs more than the overlap wins at world 1."""
        self.comm = comm
        self.overlap_comm = bool(overlap_comm)
        self.W, self.rank = comm.world, comm.rank
        self.device = torch.device(device)
        dev = self.device
        self.F = 2
        self.B = int(batch_size)
        self.D = int(embedding_dim)
        self.N = [int(n) for n in num_embeddings]
        self.layer_sizes = [int(x) for x in layer_sizes]
        self.lr_emb, self.lr_dense, self.eps = float(lr_emb), float(lr_dense), float(eps)
        self.id_dtype = id_dtype
        sharding = list(sharding or ["row_wise"] * self.F)
        tw_owners = list(tw_owners or [f % self.W for f in range(self.F)])
        self.sharding = sharding
        W, r, F, B, D = self.W, self.rank, self.F, self.B, self.D
        # ---- shards
        self.block, self.owner, local_rows, self.row_lo = [], [], [], []
        for f in range(F):
            if sharding[f] == "row_wise":
                bs = -(-self.N[f] // W)
                lo = min(r * bs, self.N[f])
                self.block.append(bs)
                self.owner.append(0)
                self.row_lo.append(lo)
                local_rows.append(max(0, min(bs, self.N[f] - lo)))
            elif sharding[f] == "table_wise":
                self.block.append(0)
                self.owner.append(int(tw_owners[f]))
                self.row_lo.append(0)
                local_rows.append(self.N[f] if tw_owners[f] == r else 0)
            else:
                raise _lib.TTError(f"sharding must be row_wise / table_wise, got {sharding[f]}")
        self.local_rows = local_rows
        self.tables = ops.TableSet([max(1, n) for n in local_rows], [D] * F, list(range(F)), dev)
        for f in range(F):
            view = self.tables.table_view(f)
            if full_tables is not None:
                if local_rows[f]:
                    lo = self.row_lo[f]
                    view[:local_rows[f]].copy_(full_tables[f][lo:lo + local_rows[f]])
            else:
                a = (1.0 / self.N[f]) ** 0.5
                view.uniform_(-a, a, generator=torch.Generator(device=dev).manual_seed(seed * 1000 + 17 * r + f))
        # ---- exchange buffers (fixed sizes)
        # a table-wise feature sends all B lookups to its owner: its segment needs capacity B
        if capacity is None:
            capacity = B if "table_wise" in sharding else default_capacity(B, W)
        self.C = int(capacity)
        C_ = self.C
        self.nslots = W * F * C_
        self.send = torch.zeros(W, F + F * C_, dtype=torch.int64, device=dev)
        self.recv = torch.zeros_like(self.send)
        self.pos = torch.full((F * B,), -1, dtype=torch.int32, device=dev)
        # gathered rows travel as bf16 (T1 computes on bf16 inputs, so nothing changes but the bytes:
        # half the rows all-to-all); gradient rows stay fp32 (the fp32 row-wise Adagrad)
        self.rows_out = torch.zeros(self.nslots, D, dtype=torch.bfloat16, device=dev)
        self.rows_in = torch.zeros_like(self.rows_out)
        self.grad_out = torch.zeros(self.nslots, D, dtype=torch.float32, device=dev)
        self.grad_in = torch.zeros_like(self.grad_out)
        self.flags = torch.zeros(2, dtype=torch.int32, device=dev)  # {overflow, bad key}
        self.route_ws = torch.empty(_lib.load().tt_shard_route_workspace_bytes(F, B), dtype=torch.uint8, device=dev)
        self.tables.ensure_dedup_workspace(self.nslots)
        # ---- towers (data-parallel replicas)
        if not ops.FusedTowers.supported([D, D], self.layer_sizes, [0, D], B) or len(self.layer_sizes) != 2 or D > 128:
            raise _lib.TTError("sharded step: towers must be 2 layers with D <= 128 (fused T1 indexed mode)")
        self.towers = ops.FusedTowers([D, D], self.layer_sizes, [0, D], B, dev)
        n = self.towers.num_params
        self.params = torch.empty(n, dtype=torch.float32, device=dev)
        self.grads = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.adam_state = torch.zeros(2, dtype=torch.int64, device=dev)
        g = torch.Generator().manual_seed(seed + 1)
        chunks, o = [], 0
        for _ in range(2):
            i = D
            for out in self.layer_sizes:
                bound = 1.0 / i ** 0.5
                w = torch.empty(out, i).uniform_(-bound, bound, generator=g)
                b = torch.empty(out).uniform_(-bound, bound, generator=g)
                chunks += [w.flatten(), b]
                i = out
        self.params.copy_(torch.cat(chunks))
        self.towers.update(self.params, do_adam=False)
        # ---- step inputs / outputs
        self.cols = [torch.zeros(B, dtype=id_dtype, device=dev) for _ in range(F)]
        self.labels = torch.zeros(B, dtype=torch.int32, device=dev)
        self.logits = torch.empty(B, dtype=torch.float32, device=dev)
        self.loss = torch.zeros((), dtype=torch.float32, device=dev)
        self._ne = (C.c_int64 * F)(*self.N)
        self._bs = (C.c_int64 * F)(*self.block)
        self._ow = (C.c_int32 * F)(*self.owner)
        self.pool_graphs: list = []

    # ------------------------------------------------------------------------------------------
    def layer_views(self):
        """[(W, b)] per tower (query, candidate) as views of the flat parameter buffer."""
        out, o, D = [], 0, self.D
        for _ in range(2):
            layers, i = [], D
            for n in self.layer_sizes:
                w = self.params[o:o + n * i].view(n, i)
                o += n * i
                b = self.params[o:o + n]
                o += n
                layers.append((w, b))
                i = n
            out.append(layers)
        return out

    def load_batch(self, cols: Sequence[torch.Tensor], labels: torch.Tensor) -> None:
        for dst, src in zip(self.cols, cols):
            dst.copy_(src, non_blocking=True)
        self.labels.copy_(labels, non_blocking=True)

    def step(self) -> None:
        lib = _lib.load()
        st = stream_handle(self.device)
        F, B, W, C_ = self.F, self.B, self.W, self.C
        ts, tw = self.tables, self.towers
        # input_dist: route + ids all-to-all
        check(lib.tt_shard_route_cols(F, B, ptr_array(list(self.cols)), id_dtype_code(self.cols[0].dtype), self._ne,
                                      self._bs, self._ow, W, C_, ptr(self.send), ptr(self.pos), ptr(self.flags),
                                      ptr(self.route_ws), self.route_ws.numel(), st),
              "shard_route_cols")
        self.comm.all_to_all(self.recv, self.send)
        # owner lookup (+ dedup insert), rows back
        check(lib.tt_shard_gather_rows_bf16(ptr(ts.weights), ts._tm, ts.T, F, W, C_, ptr(self.recv),
                                            ptr(self.rows_out), ptr(self.flags[1:]), ptr(ts._dd_ws), ts._dd_ws.numel(),
                                            ts._dd_cap, st),
              "shard_gather_rows")
        self.comm.all_to_all(self.rows_in, self.rows_out)
        # towers (dX straight into the gradient rows the owners receive)
        tw.fwd_bwd_indexed([self.pos[:B], self.pos[B:]], [self.rows_in, self.rows_in],
                           [self.grad_out, self.grad_out], self.params, self.labels, self.logits)
        # gradient rows to the owners (with overlap_comm: beside the towers' weight gradients (T2)
        # and their reduction, and the towers' all-reduce beside the owner's row-wise Adagrad)
        h_rows = self.comm.all_to_all(self.grad_in, self.grad_out, async_op=self.overlap_comm)
        tw.wgrad(self.loss)
        tw.update(self.params, do_adam=False, grads_out=self.grads)
        h_dense = self.comm.all_reduce_mean(self.grads, async_op=self.overlap_comm)
        h_rows.wait()
        ts.dedup_rowwise_adagrad(self.grad_in, self.nslots, self.lr_emb, self.eps, flat=True)
        h_dense.wait()
        tw.adam_grads(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.adam_state, lr=self.lr_dense)

    # ---- checkpoint (03_model_training.py:474-502 / :1015-1054 format) -------------------------
    def spans(self, f: int) -> List[Tuple[int, int]]:
        """(first row, rows) of table f held by each rank."""
        out = []
        for r in range(self.W):
            if self.sharding[f] == "row_wise":
                bs = self.block[f]
                lo = min(r * bs, self.N[f])
                out.append((lo, max(0, min(bs, self.N[f] - lo))))
            else:
                out.append((0, self.N[f] if self.owner[f] == r else 0))
        return out

    def gathered_state_dict(self, feature_names: Sequence[str] = ("user_id", "product_id"),
                            prefix: str = "two_tower.") -> Dict[str, torch.Tensor]:
        """Collective: rank 0 returns the full state dict the reference's gather_and_get_state_dict
        writes (full tables + towers), other ranks {}."""
        from .lifecycle import _dense_items, _tower_views

        sd = {}
        for f, name in enumerate(feature_names):
            full = self.comm.gather_rows(self.tables.table_view(f), self.spans(f), self.N[f])
            if self.rank == 0:
                sd[f"{prefix}ebc.embedding_bags.t_{name}.weight"] = full
        if self.rank == 0:
            towers = _tower_views(self.params, [self.D, self.D], self.layer_sizes)
            sd.update({k: v.clone() for k, v in _dense_items(towers, prefix).items()})
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor], feature_names: Sequence[str] = ("user_id", "product_id"),
                        prefix: str = "two_tower.") -> None:
        """Every rank takes its blocks of the full tables and the towers from a gathered dict."""
        from .lifecycle import _dense_items, _tower_views

        with torch.no_grad():
            for f, name in enumerate(feature_names):
                lo, n = self.spans(f)[self.rank]
                if n:
                    self.tables.table_view(f)[:n].copy_(sd[f"{prefix}ebc.embedding_bags.t_{name}.weight"][lo:lo + n])
            towers = _tower_views(self.params, [self.D, self.D], self.layer_sizes)
            for k, v in _dense_items(towers, prefix).items():
                v.copy_(sd[k])
        self.towers.update(self.params, do_adam=False)

    def check(self) -> None:
        """Raise if any step so far overflowed a segment or received a key outside its shard."""
        f = self.flags.cpu().tolist()
        if f[0]:
            raise _lib.TTError(f"sharded step: a segment exceeded its capacity C={self.C} (skewed ids): "
                               "results are invalid; raise `capacity`")
        if f[1]:
            raise _lib.TTError("sharded step: an owner received a key outside its shard")

    def release_graphs(self) -> None:
        """Drop the captured graphs (call before tearing down the process group: a live graph
        holds references to the RCCL communicator's work)."""
        torch.cuda.synchronize(self.device)
        self.pool_graphs = []
        self._pool_inputs = []
        import gc

        gc.collect()
        torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------------------------------
    def capture_pool(self, batches: Sequence, steps_per_graph: int = 1) -> None:
        """HIP graphs over resident (cols, labels) batches, k steps per graph (RCCL collectives
        inside; needs a capturable comm)."""
        if not self.comm.capturable:
            raise _lib.TTError("capture_pool: the comm is not graph-capturable")
        k = int(steps_per_graph)
        if k < 1 or len(batches) % k:
            raise _lib.TTError("capture_pool: the batch count must be a multiple of steps_per_graph")
        staged = [(list(c), l.to(torch.int32).contiguous()) for c, l in batches]
        self._pool_inputs = getattr(self, "_pool_inputs", []) + [staged]
        keep = self.cols, self.labels
        self.pool_graphs = []
        torch.cuda.synchronize(self.device)
        for j in range(0, len(staged), k):
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    for cols, labels in staged[j:j + k]:
                        self.cols, self.labels = cols, labels
                        self.step()
            torch.cuda.current_stream(self.device).wait_stream(s)
            self.pool_graphs.append(g)
        self.cols, self.labels = keep
        torch.cuda.synchronize(self.device)
        self.steps_per_graph = k
