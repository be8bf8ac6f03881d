"""The whole two-tower training step on one MI355X as a fixed sequence of libtt_mi355x launches,
replayable as one HIP graph.

Semantics = one ``TrainPipelineSparseDist.progress`` of the reference (03_model_training.py:618)
over ``transform_to_torchrec_batch`` (:353-382), ``TwoTowerTrainTask(TwoTower(ebc, layer_sizes))``
(:395-455), RowWiseAdagrad applied in backward to the tables (:791-795) and Adam on the towers
(:826-829) — with the reference's host KJT loop replaced by the device KJT builder and every
intermediate kept in place:

  side stream:  k2a-c  bwd_prepare (hash/count/scan/scatter)   <- depends on the ids only
  main stream:  kjt_build -> pooled_fwd -> towers fwd (grouped bf16 MFMA, both towers per launch,
                layer 0 reads the KeyedTensor column slices in place) -> dot+BCE(+grad)
                -> towers bwd (dX into the pooled-gradient slices, dW/db split-K)
                -> [join] k2d fused row-wise Adagrad -> Adam on the flat dense buffer

No host synchronisation inside ``step()``: buffers are sized for the worst case (every id kept).
"""
from __future__ import annotations


from typing import List, Optional, Sequence

import ctypes as C

import torch

from . import _lib, ops
from ._lib import FeatureMeta, check, id_dtype_code, ptr, ptr_array, stream_handle


class FusedTwoTowerStep:
    def __init__(self, num_embeddings: Sequence[int], embedding_dims: Sequence[int],
                 query_features: Sequence[int], candidate_features: Sequence[int], layer_sizes: Sequence[int],
                 batch_size: int, device: torch.device, lr_emb: float = 0.01, lr_dense: float = 0.01,
                 eps: float = 1e-10, id_dtype: torch.dtype = torch.int64, seed: int = 0,
                 overlap_prepare: bool = True, precision: str = "bf16", fused_towers: bool = True,
                 kjt_mode: str = "cols", overlap_towers: bool = True, fuse_gather: bool = True,
                 materialize_pooled: bool = False, dedup: str = "single", combined_bwd: bool = True,
                 max_lookups: Optional[int] = None, tables: Optional[ops.TableSet] = None):
        """One table per feature (feature f -> table f), features ordered as the KJT keys.
        precision: tower GEMM operands "bf16" (production) or "fp32" (parity mode).
        overlap_prepare / overlap_towers: run the dedup prepare / the towers' weight-gradient and
        Adam kernels on side streams (False: everything in order on the caller's stream).
        fuse_gather: with single-hot columns, one key per tower and two-layer towers, the EBC
        forward runs inside the tower kernel (rows gathered straight into its LDS tile); the
        pooled rows are then written to ``self.pooled`` only when ``materialize_pooled``.
        dedup: "single" — single-hot columns use the two-launch dedup (csrc/dedup.hip: the insert
        fused into the tower kernel, one update launch); "kjt" — the KJT-form hash/scan/scatter
        kernels (always used in kjt_mode "kjt").
        combined_bwd: with the fused gather and the single-hot dedup, run the whole step on ONE
        stream as three launches — T1 (gather + towers + dedup insert), T2 + row-wise Adagrad in
        one launch, T3 (Adam) — instead of side streams (cross-stream joins inside a HIP graph
        cost several microseconds each).
        max_lookups: multi-hot KJT input (config 5 bags): the step takes a KeyedJaggedTensor's
        values / offsets through ``load_kjt`` (ids already in range, as TorchRec's EBC takes them) with
        up to ``max_lookups`` ids per step, and runs the KJT-form kernels (tt_pooled_fwd, tiled
        tt_bwd_prepare, tt_bwd_rowwise_adagrad) around the fused towers.
        tables: adopt an existing TableSet (table f = feature f's; e.g. an EmbeddingBagCollection's or
        a one-rank ShardedEmbeddingBagCollection's storage): the step trains those weights and that
        row-wise Adagrad state in place and initialises neither (dropin.py)."""
        self.device = torch.device(device)
        self.precision = precision
        if kjt_mode not in ("cols", "kjt"):
            raise _lib.TTError("kjt_mode must be 'cols' or 'kjt'")
        self.kjt_input = max_lookups is not None
        if self.kjt_input:
            kjt_mode = "kjt"
        self.kjt_mode = kjt_mode
        self.offsets_used = None
        self.F = len(num_embeddings)
        self.B = int(batch_size)
        self.num_embeddings = [int(n) for n in num_embeddings]
        self.dims = [int(d) for d in embedding_dims]
        self.qf = list(query_features)
        self.cf = list(candidate_features)
        self.layer_sizes = [int(x) for x in layer_sizes]
        self.lr_emb, self.lr_dense, self.eps = float(lr_emb), float(lr_dense), float(eps)
        self.id_dtype = id_dtype
        dev = self.device
        self.out_dim = sum(self.dims)
        col = [0]
        for d in self.dims:
            col.append(col[-1] + d)
        self.col = col
        # tables (one flat HBM buffer) + row-wise state
        self._adopted = tables is not None
        if self._adopted:
            if tables.T < self.F or [tables.rows[f] for f in range(self.F)] != self.num_embeddings or \
                    [tables.dims[f] for f in range(self.F)] != self.dims or tables.device != dev:
                raise _lib.TTError("fused step: the adopted TableSet's tables must be feature f -> table f with "
                                   "the step's rows, dims and device")
            self.tables = tables.remap(list(range(self.F)), col[:-1])
        else:
            self.tables = ops.TableSet(self.num_embeddings, self.dims, list(range(self.F)), dev)
            gen = torch.Generator(device=dev).manual_seed(seed)
            self.tables.init_uniform_(gen)
        # the reference's towers take the concatenation of their features; with the KJT key order
        # (query features, then candidate features) each tower input is one contiguous column slice
        self.q_lo, self.q_hi = col[min(self.qf)], col[max(self.qf) + 1]
        self.c_lo, self.c_hi = col[min(self.cf)], col[max(self.cf) + 1]
        if sorted(self.qf) != list(range(min(self.qf), max(self.qf) + 1)) or \
                sorted(self.cf) != list(range(min(self.cf), max(self.cf) + 1)):
            raise _lib.TTError("fused step: tower features must be contiguous KJT keys")
        self.in_q = self.q_hi - self.q_lo
        self.in_c = self.c_hi - self.c_lo
        # dense parameters: one flat fp32 buffer (towers' W, b), grads and Adam moments beside it
        shapes = []
        for tower_in in (self.in_q, self.in_c):
            i = tower_in
            for o in self.layer_sizes:
                shapes.append((o, i))
                shapes.append((o,))
                i = o
        n = sum(torch.Size(s).numel() for s in shapes)
        self.params = torch.empty(n, dtype=torch.float32, device=dev)
        self.grads = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.adam_state = torch.zeros(2, dtype=torch.int64, device=dev)
        views, gviews, o = [], [], 0
        for s in shapes:
            k = torch.Size(s).numel()
            views.append(self.params[o:o + k].view(s))
            gviews.append(self.grads[o:o + k].view(s))
            o += k
        L = len(self.layer_sizes)
        self.qW = [views[2 * l] for l in range(L)]
        self.qb = [views[2 * l + 1] for l in range(L)]
        self.cW = [views[2 * L + 2 * l] for l in range(L)]
        self.cb = [views[2 * L + 2 * l + 1] for l in range(L)]
        self.gqW = [gviews[2 * l] for l in range(L)]
        self.gqb = [gviews[2 * l + 1] for l in range(L)]
        self.gcW = [gviews[2 * L + 2 * l] for l in range(L)]
        self.gcb = [gviews[2 * L + 2 * l + 1] for l in range(L)]
        g = torch.Generator().manual_seed(seed + 1)
        for W_, b_ in list(zip(self.qW, self.qb)) + list(zip(self.cW, self.cb)):
            bound = 1.0 / W_.shape[1] ** 0.5  # nn.Linear default init
            W_.copy_(torch.empty(W_.shape).uniform_(-bound, bound, generator=g))
            b_.copy_(torch.empty(b_.shape).uniform_(-bound, bound, generator=g))
        self.grouped = self.in_q == self.in_c
        # static step buffers
        B, F = self.B, self.F
        self.cols = [torch.zeros(B, dtype=id_dtype, device=dev) for _ in range(F)]
        self.labels = torch.zeros(B, dtype=torch.int32, device=dev)
        self.max_lookups = int(max_lookups) if self.kjt_input else F * B
        self.values = torch.zeros(max(1, self.max_lookups), dtype=id_dtype, device=dev)
        self.lengths = torch.zeros(F * B, dtype=torch.int32, device=dev)
        self.offsets = torch.zeros(F * B + 1, dtype=torch.int32, device=dev)
        self.lpk = torch.empty(F, dtype=torch.int64, device=dev)
        self.pooled = torch.empty(B, self.out_dim, dtype=torch.float32, device=dev)
        self.gpooled = torch.empty(B, self.out_dim, dtype=torch.float32, device=dev)
        self.qy = [torch.empty(B, n_, dtype=torch.float32, device=dev) for n_ in self.layer_sizes]
        self.cy = [torch.empty(B, n_, dtype=torch.float32, device=dev) for n_ in self.layer_sizes]
        self.qdy = [torch.empty(B, n_, dtype=torch.float32, device=dev) for n_ in self.layer_sizes]
        self.cdy = [torch.empty(B, n_, dtype=torch.float32, device=dev) for n_ in self.layer_sizes]
        self.logits = torch.empty(B, dtype=torch.float32, device=dev)
        self.loss = torch.zeros((), dtype=torch.float32, device=dev)
        self.dot_bce = ops.DotBCE(dev, B)
        self.tables.ensure_bwd_workspace(self.max_lookups)
        self.side = torch.cuda.Stream(device=dev) if overlap_prepare else None
        # multi-hot step: the rows looked up more than once (tt_bwd_rowwise_adagrad_part 2) on their
        # own stream beside the once-looked-up rows' update (part 1, the step's critical path:
        # 378-380 against 382-384 µs on one stream)
        self.side3 = torch.cuda.Stream(device=dev) if overlap_prepare else None
        # multi-hot pipelined step: the next batch's grouping is joined by the NEXT step's update
        # (it may run on beside that step's T1) instead of at this step's end (383 against 388-391 µs)
        self.cross_step_grouping = True
        self._prep_event = None
        # bf16 towers on the three fused kernels when the shape allows (else per-layer GEMMs)
        self.towers = None
        if precision == "bf16" and fused_towers and ops.FusedTowers.supported(
                [self.in_q, self.in_c], self.layer_sizes, [self.q_lo, self.c_lo], B):
            self.towers = ops.FusedTowers([self.in_q, self.in_c], self.layer_sizes, [self.q_lo, self.c_lo], B, dev)
            assert self.towers.num_params == self.params.numel()
            self.side2 = torch.cuda.Stream(device=dev) if overlap_towers else None
            self.sync_weights()
        if dedup not in ("single", "kjt"):
            raise _lib.TTError("dedup must be 'single' or 'kjt'")
        self.dedup_single = dedup == "single" and kjt_mode == "cols" and max(self.dims) <= 128 and \
            all(d % 4 == 0 for d in self.dims)
        if self.dedup_single:
            self.tables.ensure_dedup_workspace(F * B)
        self.materialize_pooled = bool(materialize_pooled)
        # ring: tower_l2_kernel's dedup wave touches the next batch's rows after its own gather (cache
        # / TLB prefetch); the row-owned T1 touches nothing (there the touches' TLB misses stall the
        # workgroup's later stores, and beside T3 they cost T3 more than they save T1: DESIGN.md
        # section 3)
        self.prefetch_next = True
        # ring: T2 + complete next-batch insert + update of the rows looked up more than once in one
        # launch, then T3 alone (False, tests: T2 + deferred insert, then resolver + update + T3)
        self.ring_tail = True
        self.combined_bwd = bool(combined_bwd)
        # in-graph kernel timing (bench): while a list, step() records an event pair per launch
        self._timing: Optional[list] = None
        self.gather = (fuse_gather and self.towers is not None and kjt_mode == "cols" and self.F == 2
                       and self.qf == [0] and self.cf == [1] and len(self.layer_sizes) == 2
                       and max(self.dims) <= 128)
        # multi-hot KJT input: the EBC forward (sum pool of every bag) runs inside T1
        # (tt_tower_fwd_bwd_kjt) for one key per tower, towers [128, 64] over 64- or 128-wide rows
        # (fuse_gather=False: tt_pooled_fwd + T1 on the pooled rows)
        self.gather_kjt = (fuse_gather
                           and self.towers is not None and self.kjt_input and self.F == 2
                           and self.qf == [0] and self.cf == [1] and self.layer_sizes == [128, 64]
                           and self.dims[0] == self.dims[1] and self.dims[0] in (64, 128))
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        # warm every scratch workspace so graph capture allocates nothing new (the all-zero batch
        # drops every id, so the tables are untouched; the towers' parameters are restored)
        p0 = self.params.clone()
        self.step()
        torch.cuda.synchronize(dev)
        self.params.copy_(p0)
        self.sync_weights()
        self.reset_optimizer_state()

    # ------------------------------------------------------------------------------------------
    def reset_optimizer_state(self) -> None:
        if not self._adopted:  # an adopted TableSet keeps its owner's row-wise Adagrad state
            self.tables.state.zero_()
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()
        self.adam_state.zero_()

    def load_batch(self, cols: Sequence[torch.Tensor], labels: torch.Tensor) -> None:
        for dst, src in zip(self.cols, cols):
            dst.copy_(src, non_blocking=True)
        self.labels.copy_(labels, non_blocking=True)

    def load_kjt(self, values: torch.Tensor, offsets: torch.Tensor, labels: torch.Tensor) -> None:
        """Multi-hot input (``max_lookups`` set): a KJT's values (keys in step order, key-major bags)
        and its complete offsets [F*B + 1] (int32), plus labels. Copied into the step's static
        buffers (graph-capturable)."""
        if not self.kjt_input:
            raise _lib.TTError("load_kjt: construct the step with max_lookups")
        n = values.numel()
        if n > self.max_lookups or offsets.numel() != self.F * self.B + 1:
            raise _lib.TTError("load_kjt: more ids than max_lookups, or offsets not [F*B + 1]")
        self.values[:n].copy_(values, non_blocking=True)
        self.offsets.copy_(offsets.to(torch.int32), non_blocking=True)
        self.labels.copy_(labels, non_blocking=True)

    def capture_pool_kjt(self, batches: Sequence, keep_graph: bool = False, ahead: bool = False,
                         steps_per_graph: int = 1) -> None:
        """One graph per resident multi-hot batch (values, offsets int32, labels), read in place.
        ahead: the pipelined form (``step(next_kjt=...)``): graph i groups batch i+1 of the pool
        while it trains on batch i, so the graphs must be replayed in pool order from the cursor
        (``replay_pool``); the pool length must be even (the two grouping workspaces alternate).
        steps_per_graph k > 1 (ahead only; the pool length a multiple of k): also graphs of k
        consecutive steps (``pool_graphs_k``), which ``replay_pool`` uses where the cursor allows —
        between two graphs the stream idles ~20 us (the step's side branches join, the next graph
        launches); inside one graph the next step's T1 follows the join directly."""
        staged = []
        for values, offsets, labels in batches:
            if values.dtype != self.id_dtype or offsets.dtype != torch.int32 or values.numel() > self.max_lookups \
                    or offsets.numel() != self.F * self.B + 1:
                raise _lib.TTError("capture_pool_kjt: batch does not match the step's dtype / capacity")
            staged.append((values.contiguous(), offsets.contiguous(), labels.to(torch.int32).contiguous()))
        n = len(staged)
        k = int(steps_per_graph)
        if ahead and n % 2:
            raise _lib.TTError("capture_pool_kjt(ahead=True): the batch count must be even")
        if k > 1 and (not ahead or n % k or k % 2):
            raise _lib.TTError("capture_pool_kjt: steps_per_graph > 1 needs ahead=True, an even k dividing the pool")
        self._prefault_due = True  # the next replay walks the tables' pages first (TableSet.prefault)
        self._pool_inputs = getattr(self, "_pool_inputs", []) + [staged]
        keep = self.values, self.offsets, self.labels
        self.pool_graphs = []
        self.pool_graphs_k = []
        self.pool_mid = {}
        self.pool_offset = 0
        self.pool_ahead = bool(ahead)
        self._kjt_pool = staged
        self._kjt_keep_graph = keep_graph
        if ahead:
            self.kjt_ring_prime(staged[0][0], staged[0][1], 0)
        self.steps_per_graph = k
        try:
            for i in range(n):
                self.pool_graphs.append(self._capture_kjt_steps([self._kjt_item(i)], keep_graph))
        finally:
            self.values, self.offsets, self.labels = keep
        self._kjt_groups(0)
        self.graph = self.pool_graphs[-1]
        self.pool_cursor = 0

    def _kjt_item(self, i):
        """(values, offsets, labels, next batch's KJT or None, parity) of pool position i."""
        staged, n = self._kjt_pool, len(self._kjt_pool)
        v, o, lab = staged[i]
        nxt = (staged[(i + 1) % n][0], staged[(i + 1) % n][1]) if self.pool_ahead else None
        return v, o, lab, nxt, i % 2

    def _kjt_groups(self, offset: int) -> None:
        """The multi-step pool graphs grouped from pool position ``offset``: k-step graphs and (k a
        power of two) k/2, ..., 2-step ones at the same alignment, so a run replays few graph
        launches (a graph ends by joining its last step's side branches and the next one launches:
        the stream idles ~20-40 us between two graphs, which single-step graphs pay every step)."""
        n, k = len(self._kjt_pool), self.steps_per_graph
        self.pool_offset = offset % n
        self.pool_graphs_k, self.pool_mid = [], {}
        if k < 2:
            return
        keep = self.values, self.offsets, self.labels
        span = lambda j, sz: [self._kjt_item((offset + j + t) % n) for t in range(sz)]  # noqa: E731
        try:
            kg = self._kjt_keep_graph
            self.pool_graphs_k = [self._capture_kjt_steps(span(j, k), kg, sync=False) for j in range(0, n, k)]
            sz = k // 2 if k & (k - 1) == 0 else 0
            while sz >= 2:
                self.pool_mid[sz] = [self._capture_kjt_steps(span(j, sz), kg, sync=False) for j in range(0, n, sz)]
                sz //= 2
        finally:
            self.values, self.offsets, self.labels = keep

    def align_pool(self, n_next: int = 0, after: int = 0) -> None:
        """Regroup the multi-step pool graphs for a run of ``n_next`` steps that starts ``after``
        steps from the cursor (the training state is untouched: only how the steps are grouped into
        graph launches changes): the run replays its n_next % k remainder first, in aligned smaller
        graphs, then n_next // k full graphs. Call it before the warm-up that precedes the run."""
        k, n = self.steps_per_graph, len(self.pool_graphs)
        off = (self.pool_cursor + after + (n_next % k)) % n
        if k > 1 and off != self.pool_offset:
            self._kjt_groups(off)

    def _capture_kjt_steps(self, items, keep_graph: bool, sync: bool = True):
        """One HIP graph of consecutive multi-hot steps; items: (values, offsets, labels, next_kjt,
        parity) per step. sync: refresh the bf16 weight copies first (not when regrouping mid-run)."""
        if sync:
            self.sync_weights()
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph(keep_graph=keep_graph)
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for v, o, lab, nxt, par in items:
                    self.values, self.offsets, self.labels = v, o, lab
                    self.step(next_kjt=nxt, parity=par)
                self.kjt_join()  # every forked stream rejoins inside the graph
        torch.cuda.current_stream(self.device).wait_stream(s)
        if not keep_graph:
            _lib.graph_upload(g, self.device)
        torch.cuda.synchronize(self.device)
        return g

    def kjt_join(self) -> None:
        """Make the current stream wait for the next batch's grouping a pipelined multi-hot step left
        running on the side stream (the following step joins it before its update; a captured graph
        and any other use join it here)."""
        ev = getattr(self, "_prep_event", None)
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
            self._prep_event = None

    def kjt_ring_prime(self, values: torch.Tensor, offsets: torch.Tensor, parity: int) -> None:
        """Group the first batch of a pipelined multi-hot sequence into workspace ``parity`` (every
        later batch is grouped by the step before it)."""
        ts = self.tables
        ts.use_bwd_workspace(1 - parity)  # both workspaces exist before any graph capture
        ts.use_bwd_workspace(parity)
        ts.bwd_prepare(values, offsets, self.B, max_lookups=self.max_lookups)

    def replay_pool(self, n: int) -> None:
        """Replay n pool graphs in pool order, continuing at the cursor (the pipelined pool needs
        the order: graph i expects batch i's grouping from graph i-1)."""
        if getattr(self, "_prefault_due", False):  # first replay after a capture: the tables' pages
            self._prefault_due = False  # walked right before it (TableSet.prefault; r06pf_* profiles)
            self.tables.prefault()
        i, nb = self.pool_cursor, len(self.pool_graphs)
        k = getattr(self, "steps_per_graph", 1)
        mid = getattr(self, "pool_mid", {})
        off = getattr(self, "pool_offset", 0)
        while n > 0:
            r = (i - off) % nb  # position relative to the multi-step graphs' grouping
            if k > 1 and self.pool_graphs_k and r % k == 0 and n >= k:
                self.pool_graphs_k[r // k].replay()
                sz = k
            else:
                sz = next((m for m in sorted(mid, reverse=True) if r % m == 0 and n >= m), 1)
                (mid[sz][r // sz] if sz > 1 else self.pool_graphs[i]).replay()
            i, n = (i + sz) % nb, n - sz
        self.pool_cursor = i

    def pool_step_eager(self) -> None:
        """One step of the captured multi-hot pool at the cursor without graphs (timing / tests)."""
        staged, i = self._kjt_pool, self.pool_cursor
        n = len(staged)
        keep = self.values, self.offsets, self.labels
        self.values, self.offsets, self.labels = staged[i]
        try:
            if self.pool_ahead:
                self.step(next_kjt=(staged[(i + 1) % n][0], staged[(i + 1) % n][1]), parity=i % 2)
            else:
                self.step()
        finally:
            self.values, self.offsets, self.labels = keep
        self.pool_cursor = (i + 1) % n

    def _towers_fwd(self):
        L = len(self.layer_sizes)
        pr = self.precision
        xq = self.pooled[:, self.q_lo:self.q_hi]
        xc = self.pooled[:, self.c_lo:self.c_hi]
        for l in range(L):
            if self.grouped:
                ops.linear_fwd([xq, xc], [self.qW[l], self.cW[l]], [self.qb[l], self.cb[l]], relu=True,
                               outs=[self.qy[l], self.cy[l]], precision=pr)
            else:
                ops.linear_fwd([xq], [self.qW[l]], [self.qb[l]], relu=True, outs=[self.qy[l]], precision=pr)
                ops.linear_fwd([xc], [self.cW[l]], [self.cb[l]], relu=True, outs=[self.cy[l]], precision=pr)
            xq, xc = self.qy[l], self.cy[l]

    def _towers_bwd(self):
        L = len(self.layer_sizes)
        pr = self.precision
        for l in reversed(range(L)):
            xq = self.pooled[:, self.q_lo:self.q_hi] if l == 0 else self.qy[l - 1]
            xc = self.pooled[:, self.c_lo:self.c_hi] if l == 0 else self.cy[l - 1]
            dxq = self.gpooled[:, self.q_lo:self.q_hi] if l == 0 else self.qdy[l - 1]
            dxc = self.gpooled[:, self.c_lo:self.c_hi] if l == 0 else self.cdy[l - 1]
            if self.grouped:
                ops.linear_bwd_data([self.qdy[l], self.cdy[l]], [self.qy[l], self.cy[l]], [self.qW[l], self.cW[l]],
                                    relu=True, outs=[dxq, dxc], precision=pr)
                ops.linear_bwd_weight([self.qdy[l], self.cdy[l]], [self.qy[l], self.cy[l]], [xq, xc], relu=True,
                                      dws=[self.gqW[l], self.gcW[l]], dbs=[self.gqb[l], self.gcb[l]], precision=pr)
            else:
                for dy, y, W_, x, dx, gW, gb in ((self.qdy[l], self.qy[l], self.qW[l], xq, dxq, self.gqW[l], self.gqb[l]),
                                                 (self.cdy[l], self.cy[l], self.cW[l], xc, dxc, self.gcW[l], self.gcb[l])):
                    ops.linear_bwd_data([dy], [y], [W_], relu=True, outs=[dx], precision=pr)
                    ops.linear_bwd_weight([dy], [y], [x], relu=True, dws=[gW], dbs=[gb], precision=pr)

    def step(self, next_kjt: Optional[Sequence[torch.Tensor]] = None, parity: int = 0) -> None:
        """One training step on the batch currently in ``cols`` / ``labels`` (multi-hot: ``values`` /
        ``offsets`` / ``labels``).
        next_kjt (multi-hot input only): the pipelined form. This batch's backward grouping is
        already complete in grouping workspace ``parity`` (built by the previous step, or by
        ``kjt_ring_prime``); the grouping of next_kjt = (values, offsets) is built into workspace
        1 - parity on the side stream, beside this step's forward, towers and update."""
        B, F = self.B, self.F
        main = torch.cuda.current_stream(self.device)
        ahead = next_kjt is not None
        if not ahead:
            self.kjt_join()
        if ahead and not (self.kjt_input and self.side is not None):
            raise _lib.TTError("step(next_kjt): needs multi-hot input (max_lookups) and overlap_prepare")
        if self.kjt_mode == "kjt":
            # materialise the KJT (values / lengths / offsets) from the single-hot columns, or take
            # the multi-hot KJT as loaded; then the KJT-form kernels
            if not self.kjt_input:
                ops.kjt_build_mod_dropzero(self.cols, self.num_embeddings, self.values, self.lengths, self.offsets,
                                           self.lpk)
            if ahead:
                ts = self.tables

                def prepare():
                    ts.use_bwd_workspace(1 - parity)
                    ts.bwd_prepare(next_kjt[0], next_kjt[1], B, max_lookups=self.max_lookups)
                    ts.use_bwd_workspace(parity)
            else:
                prepare = lambda: self.tables.bwd_prepare(self.values, self.offsets, B,  # noqa: E731
                                                          max_lookups=self.max_lookups)
            self.offsets_used = self.offsets
        elif self.dedup_single:
            # single-hot columns, two-launch dedup: the insert runs inside T1 (gather) or here
            prepare = None if self.gather else (lambda: self.tables.dedup_insert_cols(self.cols, self.num_embeddings))
            self.offsets_used = None
        else:
            # single-hot columns: the transform (drop id 0, id mod N) is applied inside the kernels
            prepare = lambda: self.tables.bwd_prepare_cols(self.cols, self.num_embeddings)  # noqa: E731
            self.offsets_used = None
        def launch_prepare():
            if self.side is not None:
                self.side.wait_stream(main)
                with torch.cuda.stream(self.side):
                    self._mark("prep", 0)
                    prepare()
                    self._mark("prep", 1)
            else:
                self._mark("prep", 0)
                prepare()
                self._mark("prep", 1)

        # the next batch's grouping beside this step's embedding update rather than beside T1: T1's
        # workgroups each take a whole CU's LDS, so the grouping kernels' workgroups would hold CUs
        # T1 waits for
        defer_prepare = ahead and self.kjt_mode == "kjt" and self.towers is not None and not self.gather
        if prepare is not None and not defer_prepare:
            launch_prepare()
        if self.gather:
            # EBC forward (and, with the single-hot dedup, its insert) fused into T1
            self._mark("t1", 0)
            self.towers.fwd_bwd_gather(self.cols, self.num_embeddings,
                                       [self.tables.table_view(0), self.tables.table_view(1)], self.gpooled,
                                       self.params, self.labels, self.logits,
                                       pooled_out=self.pooled if self.materialize_pooled else None,
                                       dedup=self.tables if self.dedup_single else None, dedup_tables=(0, 1))
        elif self.kjt_mode == "kjt" and not self.gather_kjt:
            self._mark("fwd", 0)
            self.tables.pooled_fwd(self.values, self.offsets, B, out=self.pooled)
            self._mark("fwd", 1)
        elif self.kjt_mode == "kjt":
            pass  # the sum pool runs inside T1 (below)
        else:
            self.tables.pooled_fwd_cols(self.cols, self.num_embeddings, out=self.pooled)
        if self.towers is not None and self.gather and self.dedup_single and self.combined_bwd:
            # one stream: T1 -> T2 -> [T3 + fused row-wise Adagrad]
            self._mark("t1", 1)
            self._mark("t2", 0)
            self.towers.wgrad_pre(self.loss, self.adam_state, adam_lr=self.lr_dense, dedup=self.tables)
            self._mark("t2", 1)
            self._mark("k3", 0)
            self.towers.update_pre_rowwise_adagrad(self.params, self.exp_avg, self.exp_avg_sq, self.tables,
                                                   self.gpooled, B, self.lr_emb, self.eps, grads_out=self.grads)
            self._mark("k3", 1)
            return
        if self.towers is not None:
            # T1 on the critical path; T2 + T3 (weight grads, Adam) beside the embedding update
            if self.gather_kjt or not self.gather:
                self._mark("t1", 0)
                if self.gather_kjt:
                    self.towers.fwd_bwd_kjt(self.values, self.offsets,
                                            [self.tables.table_view(0), self.tables.table_view(1)], self.gpooled,
                                            self.params, self.labels, self.logits,
                                            pooled_out=self.pooled if self.materialize_pooled else None)
                else:  # tt_pooled_fwd above, then T1 on the pooled rows
                    self.towers.fwd_bwd(self.pooled, self.gpooled, self.params, self.labels, self.logits)
                self._mark("t1", 1)
                if defer_prepare and self.side2 is not None:
                    # the row update (the step's critical path) enqueued right behind T1 on the
                    # capture stream, the two side branches forked from T1's end after it: in the
                    # graph the branches captured first started first, ~12 us apart, and the
                    # update came third
                    # this batch's grouping (the previous step's side branch, joined here rather than at
                    # that step's end: it may run on into this step's T1)
                    self.kjt_join()
                    t1_done = torch.cuda.Event()
                    t1_done.record(main)
                    self.tables.use_bwd_workspace(parity)  # (prepare() leaves it so; it runs later here)
                    self._mark("upd", 0)
                    split = (self.side3 is not None and self.offsets_used is not None
                             and all(d <= 128 and d % 4 == 0 for d in self.dims))  # the narrow path
                    if split:  # the once-looked-up rows here, the others beside them (disjoint rows)
                        self.tables.bwd_rowwise_adagrad(self.gpooled, self.offsets_used, self.B, self.lr_emb, self.eps,
                                                        part=1)
                    else:
                        self._emb_update()
                    self._mark("upd", 1)
                    branches = [(self.side, prepare), (self.side2, self._kjt_t2t3)]
                    if split:
                        branches.append((self.side3, lambda: self.tables.bwd_rowwise_adagrad(
                            self.gpooled, self.offsets_used, self.B, self.lr_emb, self.eps, part=2)))
                    for st, work in branches:
                        st.wait_event(t1_done)
                        with torch.cuda.stream(st):
                            work()
                    for st, _ in branches[1:]:
                        main.wait_stream(st)
                    if self.cross_step_grouping:  # joined by the next step's update (kjt_join)
                        self._prep_event = torch.cuda.Event()
                        self._prep_event.record(self.side)
                    else:
                        main.wait_stream(self.side)
                    return
                if defer_prepare:
                    launch_prepare()
            s2 = self.side2 if self.side2 is not None else main
            if self.side2 is not None:
                self.side2.wait_stream(main)
            with torch.cuda.stream(s2):
                self._kjt_t2t3()
            if self.side is not None and prepare is not None and not ahead:
                main.wait_stream(self.side)
            self._mark("upd", 0)
            self._emb_update()
            self._mark("upd", 1)
            if ahead:
                main.wait_stream(self.side)
            if self.side2 is not None:
                main.wait_stream(self.side2)
            return
        self._towers_fwd()
        L = len(self.layer_sizes)
        self.dot_bce(self.qy[L - 1], self.cy[L - 1], self.labels, logits=self.logits, loss=self.loss,
                     dq=self.qdy[L - 1], dc=self.cdy[L - 1])
        self._towers_bwd()
        if self.side is not None and prepare is not None and not ahead:
            main.wait_stream(self.side)
        self._emb_update()
        if ahead:
            main.wait_stream(self.side)
        ops.adam_step(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.adam_state, self.lr_dense)

    def _kjt_t2t3(self) -> None:
        """T2 (weight gradients, loss) + T3 (Adam, bf16 weight copies) of the towers."""
        self._mark("t2t3", 0)
        self.towers.wgrad(self.loss)
        self.towers.update(self.params, self.exp_avg, self.exp_avg_sq, self.adam_state, lr=self.lr_dense,
                           grads_out=self.grads)
        self._mark("t2t3", 1)

    def _mark(self, name: str, end: int) -> None:
        """Record the start (end=0) / end (end=1) HIP event of launch `name` of the current step
        on the launching stream, when per-launch timing is on (bench: eager steps)."""
        if self._timing is None or not self._timing:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self._timing[-1].setdefault(name, [None, None])[end] = ev

    def _emb_update(self) -> None:
        """EBC backward + in-backward RowWiseAdagrad (03_model_training.py:791-795) on the pooled
        gradient of this step."""
        if self.dedup_single and self.gather:
            self.tables.dedup_resolve()  # the inserts T1 deferred
        if self.dedup_single:
            self.tables.dedup_rowwise_adagrad(self.gpooled, self.B, self.lr_emb, self.eps)
        else:
            self.tables.bwd_rowwise_adagrad(self.gpooled, self.offsets_used, self.B, self.lr_emb, self.eps)

    def eval_step(self, cols: Sequence[torch.Tensor], labels: torch.Tensor):
        """Forward only (pipeline.progress in eval mode, 03_model_training.py:545): pooled lookup of
        the single-hot columns, both towers (bf16 MFMA GEMMs, or fp32 in the parity precision), dot +
        BCE. Tables and towers are not touched. Returns (mean loss, logits) device tensors."""
        B = self.B
        if cols[0].numel() != B:
            raise _lib.TTError("eval_step: batch size differs from the step's")
        self.tables.pooled_fwd_cols(list(cols), self.num_embeddings, out=self.pooled)
        self._towers_fwd()
        L = len(self.layer_sizes)
        loss = torch.empty((), dtype=torch.float32, device=self.device)
        logits = torch.empty(B, dtype=torch.float32, device=self.device)
        self.dot_bce(self.qy[L - 1], self.cy[L - 1], labels, logits=logits, loss=loss)
        return loss, logits

    def sync_weights(self) -> None:
        """Refresh the fused towers' bf16 weight copies after the fp32 parameters were changed
        outside step() (initialisation, loading a checkpoint)."""
        if self.towers is not None:
            self.towers.update(self.params, do_adam=False)

    # ---- the pipelined ring (production): dedup one step ahead, single-lookup rows in T1 ---------
    def ring_supported(self) -> bool:
        return (self.gather and self.dedup_single and self.combined_bwd and self.layer_sizes == [128, 64]
                and self.in_q == self.in_c and self.in_q in (64, 128) and self.F == 2)

    def _ring_ws(self):
        if getattr(self, "_ring", None) is None:
            if not self.ring_supported():
                raise _lib.TTError("ring: needs the fused gather + single-hot dedup path, towers [128, 64], "
                                   "inputs of 64 or 128")
            ts = self.tables
            ts.ensure_dedup_workspace(self.F * self.B)
            lib = _lib.load()
            ws1 = torch.empty_like(ts._dd_ws)
            check(lib.tt_dedup_workspace_init(ptr(ws1), ws1.numel(), ts._dd_cap, stream_handle(self.device)),
                  "dedup_workspace_init")
            self._ring = [ts._dd_ws, ws1]
            self._ring_tab = (C.c_int32 * 2)(0, 1)
            self._ring_ne = (C.c_int64 * 2)(*self.num_embeddings)
        return self._ring

    def ring_reset(self) -> None:
        """Empty both dedup tables of the ring (a staged batch's table is otherwise left filled)."""
        lib = _lib.load()
        for ws in self._ring_ws():
            check(lib.tt_dedup_workspace_init(ptr(ws), ws.numel(), self.tables._dd_cap, stream_handle(self.device)),
                  "dedup_workspace_init")

    def ring_prime(self, cols: Sequence[torch.Tensor], parity: int) -> None:
        """Build the dedup table of the first batch of a ring (every later table is built by the
        step before its batch)."""
        ws = self._ring_ws()[parity]
        ts = self.tables
        check(_lib.load().tt_dedup_insert_cols(ts._tm, ts.T, ts._fm, ts.F, self.B, ptr_array(list(cols)),
                                               id_dtype_code(cols[0].dtype), self._ring_ne, ptr(ws), ws.numel(),
                                               ts._dd_cap, stream_handle(self.device)), "dedup_insert_cols")

    def ring_step(self, cols: Sequence[torch.Tensor], labels: torch.Tensor, parity: int,
                  next_cols: Sequence[torch.Tensor]) -> None:
        """One production step on (cols, labels), whose dedup table (parity) is complete; files
        next_cols into the other table. Three launches:
          T1    gather + towers fwd/bwd + in-place row-wise Adagrad of the rows looked up once
          tail  T2 (tower weight gradients, Adam scalars) + complete insert of the next batch +
                update of the rows looked up more than once (from T1's dX)
          T3    slab reduction, Adam, bf16 weight copies
        (ring_tail False: T2 + deferred insert of the next batch, then resolver + row update + T3)."""
        lib, tw, ts, B, dev = _lib.load(), self.towers, self.tables, self.B, self.device
        ring = self._ring_ws()
        ws, wsn = ring[parity], ring[parity ^ 1]
        st = stream_handle(dev)
        self._mark("t1", 0)
        check(lib.tt_tower_fwd_bwd_gather_update(
            C.byref(tw.shape), B, ptr_array(list(cols)), id_dtype_code(cols[0].dtype), self._ring_ne,
            ptr_array([ts.table_view(0), ts.table_view(1)]), ptr_array([ts.state_view(0), ts.state_view(1)]),
            ptr(self.pooled) if self.materialize_pooled else None, self.gpooled.stride(0), ptr(self.gpooled),
            ptr(self.params), ptr(labels), _lib.TT_I32, 1.0, ptr(self.logits), self.lr_emb, self.eps, ptr(ws),
            ws.numel(), ts._dd_cap, ptr_array(list(next_cols)) if self.prefetch_next else None, ptr(tw.ws),
            tw.nbytes, st), "tower_fwd_bwd_gather_update")
        self._mark("t1", 1)
        if self.ring_tail:
            self._mark("tail", 0)
            # the tail: tower weight gradients (T2) + the next batch's complete insert + the rows
            # looked up more than once (tt_launch roles WGRAD | INSERT | ADAGRAD)
            plan = self._plan(_lib.ROLE_WGRAD | _lib.ROLE_INSERT | _lib.ROLE_ADAGRAD, ws, multi_only=1)
            plan.insert = _lib.InsertRole(next_cols=ptr_array(list(next_cols)),
                                          id_dtype=id_dtype_code(next_cols[0].dtype), num_embeddings=self._ring_ne,
                                          dedup_tables=self._ring_tab, next_dedup_ws=ptr(wsn))
            _lib.launch(plan, st, "ring tail")
            self._mark("tail", 1)
            self._mark("t3", 0)
            check(lib.tt_tower_update_pre(C.byref(tw.shape), B, ptr(self.params), ptr(self.exp_avg),
                                          ptr(self.exp_avg_sq), 1e-8, 0.9, 0.999, 0.0, ptr(self.grads), ptr(tw.ws),
                                          tw.nbytes, st), "tower_update_pre")
            self._mark("t3", 1)
            return
        self._mark("t2", 0)
        plan = self._plan(_lib.ROLE_WGRAD | _lib.ROLE_INSERT, ws)
        plan.insert = _lib.InsertRole(next_cols=ptr_array(list(next_cols)), id_dtype=id_dtype_code(next_cols[0].dtype),
                                      num_embeddings=self._ring_ne, dedup_tables=self._ring_tab, next_dedup_ws=ptr(wsn),
                                      dedup_ws_bytes=wsn.numel(), dedup_max_lookups=ts._dd_cap)
        _lib.launch(plan, st, "wgrad_pre_insert")
        self._mark("t2", 1)
        self._mark("k3", 0)
        plan = self._plan(_lib.ROLE_UPDATE | _lib.ROLE_ADAGRAD | _lib.ROLE_RESOLVE, ws, multi_only=1)
        plan.resolve = _lib.ResolveRole(dedup_ws=ptr(wsn))
        _lib.launch(plan, st, "update_pre_rowwise_adagrad_resolve")
        self._mark("k3", 1)

    def _plan(self, roles: int, ws: torch.Tensor, multi_only: int = 0) -> "_lib.LaunchPlan":
        """A tt_launch plan over this step's towers, tables and dedup workspace ``ws`` with the
        WGRAD / UPDATE / ADAGRAD roles filled (the caller adds the others)."""
        tw, ts = self.towers, self.tables
        return _lib.LaunchPlan(
            roles=roles, shape=C.pointer(tw.shape), B=self.B, workspace=ptr(tw.ws), ws_bytes=tw.nbytes,
            wgrad=_lib.WgradRole(loss=ptr(self.loss), adam_step_state=ptr(self.adam_state), adam_lr=self.lr_dense,
                                 adam_beta1=0.9, adam_beta2=0.999),
            update=_lib.UpdateRole(params=ptr(self.params), exp_avg=ptr(self.exp_avg), exp_avg_sq=ptr(self.exp_avg_sq),
                                   eps=1e-8, beta1=0.9, beta2=0.999, weight_decay=0.0, grads_out=ptr(self.grads)),
            adagrad=_lib.AdagradRole(tables=ts._tm, T=ts.T, F=ts.F, features=ts._fm, B=self.B, grad=ptr(self.gpooled),
                                     ldg=self.gpooled.stride(0), weights=ptr(ts.weights), state=ptr(ts.state),
                                     lr=self.lr_emb, eps=self.eps, dedup_ws=ptr(ws), dedup_ws_bytes=ws.numel(),
                                     dedup_max_lookups=ts._dd_cap, multi_only=multi_only))

    def capture_ring(self, batches: Sequence, steps_per_graph: int = 1, keep_graph: bool = False) -> None:
        """Production HIP graphs over a cyclic pool of resident (cols, labels) batches (len even, a
        multiple of k): ring graph j runs the steps of batches j*k .. j*k+k-1, each filing the next
        batch of the pool; ``ring_small[i]`` runs batch i alone. Replay with ``run(n)`` (the step
        keeps the cursor: the batch whose dedup table is complete)."""
        k = int(steps_per_graph)
        n = len(batches)
        if k < 1 or n % k or n % 2:
            raise _lib.TTError("capture_ring: the batch count must be even and a multiple of steps_per_graph")
        staged = []
        for cols, labels in batches:
            for c in cols:
                if c.dtype != self.id_dtype or not c.is_contiguous() or c.numel() != self.B:
                    raise _lib.TTError("capture_ring: batch columns must match the step's id dtype and batch")
            staged.append((list(cols), labels.to(torch.int32).contiguous()))
        self._ring_inputs = staged
        self._prefault_due = True  # the next replay walks the tables' pages first (TableSet.prefault)
        self.ring_reset()
        self.sync_weights()
        self.ring_prime(staged[0][0], 0)
        torch.cuda.synchronize(self.device)
        self.ring_cursor = 0
        self.ring_k = k
        self._ring_keep = keep_graph
        self.ring_small = [self._ring_graph([i]) for i in range(n)]
        self._ring_groups(0)

    def _ring_graph(self, idx) -> torch.cuda.CUDAGraph:
        """One HIP graph of the production steps of pool batches ``idx`` (in order)."""
        staged, n = self._ring_inputs, len(self._ring_inputs)
        g = torch.cuda.CUDAGraph(keep_graph=self._ring_keep)
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for i in idx:
                    self.ring_step(staged[i][0], staged[i][1], i % 2, staged[(i + 1) % n][0])
        torch.cuda.current_stream(self.device).wait_stream(s)
        if not self._ring_keep:  # keep_graph: instantiated later, by its user
            _lib.graph_upload(g, self.device)
        return g

    def _ring_groups(self, offset: int) -> None:
        """The multi-step graphs, grouped from pool position ``offset``: k-step graphs, and (k a
        power of two) k/2, k/4, ..., 2-step ones at the same alignment, so a run replays few graph
        launches (one costs the host ~35-55 us, about one step of GPU time: single-step graphs leave
        the GPU idle between them)."""
        n, k = len(self._ring_inputs), self.ring_k
        span = lambda j, sz: [(offset + j + t) % n for t in range(sz)]  # noqa: E731
        self.ring_offset = offset % n
        self.ring_graphs = [self._ring_graph(span(j, k)) for j in range(0, n, k)] if k > 1 else list(self.ring_small)
        self.ring_mid = {}
        self._prefault_due = True  # the next replay walks the tables' pages first (TableSet.prefault)
        sz = k // 2 if k & (k - 1) == 0 else 0
        while sz >= 2:
            self.ring_mid[sz] = [self._ring_graph(span(j, sz)) for j in range(0, n, sz)]
            sz //= 2
        torch.cuda.synchronize(self.device)

    def align_ring(self, n_next: int = 0, after: int = 0) -> None:
        """Regroup the multi-step graphs for a run of ``n_next`` steps that starts ``after`` steps
        from the cursor (the training state is untouched: only how the steps are grouped into graph
        launches changes): that run replays its n_next % k remainder first, in aligned smaller
        graphs (the first launch is the cheapest: the GPU starts sooner), then n_next // k full
        graphs — no single-step graphs when the remainder is a sum of the captured sizes."""
        off = (self.ring_cursor + after + (n_next % self.ring_k)) % len(self.ring_small)
        if self.ring_k > 1 and off != self.ring_offset:
            self._ring_groups(off)

    def run(self, n: int) -> None:
        """Replay n production steps from the ring, continuing at the cursor."""
        if getattr(self, "_prefault_due", False):  # first replay after a capture: the tables' pages
            self._prefault_due = False  # walked right before it (TableSet.prefault; r06pf_* profiles)
            self.tables.prefault()
        i, nb, k = self.ring_cursor, len(self.ring_small), self.ring_k
        mid = self.ring_mid
        while n > 0:
            r = (i - self.ring_offset) % nb  # position relative to the graphs' grouping
            if r % k == 0 and n >= k:
                self.ring_graphs[r // k].replay()
                sz = k
            else:
                sz = next((m for m in sorted(mid, reverse=True) if r % m == 0 and n >= m), 1)
                (mid[sz][r // sz] if sz > 1 else self.ring_small[i]).replay()
            i, n = (i + sz) % nb, n - sz
        self.ring_cursor = i

    def timed_ring(self, n: int) -> dict:
        """n eager production steps (from the cursor) with a HIP event pair around every launch;
        mean device time (ms) per launch name."""
        self._timing = []
        try:
            for _ in range(n):
                self._timing.append({})
                self.run_eager(1)
            torch.cuda.synchronize(self.device)
            acc = {}
            for m in self._timing:
                for name, (a, b) in m.items():
                    acc.setdefault(name, []).append(a.elapsed_time(b))
        finally:
            self._timing = None
        return {k: sum(v) / len(v) for k, v in acc.items()}

    def run_eager(self, n: int) -> None:
        """n production steps over the captured ring's batches without graphs (timing / tests)."""
        staged = self._ring_inputs
        nb = len(staged)
        for _ in range(n):
            i = self.ring_cursor
            self.ring_step(staged[i][0], staged[i][1], i % 2, staged[(i + 1) % nb][0])
            self.ring_cursor = (i + 1) % nb

    # ------------------------------------------------------------------------------------------
    def capture(self, batches: Optional[Sequence] = None, keep_graph: bool = False,
                next_kjt: Optional[Sequence[torch.Tensor]] = None, parity: int = 0) -> None:
        """Record ``step()`` into a HIP graph (replayed by ``replay()``). With ``batches`` (a list of
        resident (cols, labels) device batches) the graph holds one full step per batch, in order."""
        self.sync_weights()
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph(keep_graph=keep_graph)
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        keep_cols, keep_labels = self.cols, self.labels
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                if batches is None:
                    self.step(next_kjt=next_kjt, parity=parity)
                else:
                    for cols, labels in batches:
                        self.cols, self.labels = list(cols), labels
                        self.step()
        self.cols, self.labels = keep_cols, keep_labels
        torch.cuda.current_stream(self.device).wait_stream(s)
        if not keep_graph:
            _lib.graph_upload(g, self.device)
        torch.cuda.synchronize(self.device)
        self.graph = g

    def replay(self, i: Optional[int] = None) -> None:
        """Replay the single-step graph, or pool graph ``i`` (which runs ``steps_per_graph`` steps)."""
        if getattr(self, "_prefault_due", False):  # first replay after a capture: the tables' pages
            self._prefault_due = False  # walked right before it (TableSet.prefault; r06pf_* profiles)
            self.tables.prefault()
        if i is None:
            self.graph.replay()
        else:
            self.pool_graphs[i % len(self.pool_graphs)].replay()

    def timed_steps(self, batches: Sequence, n: int) -> dict:
        """Run n eager steps over the resident batches with a HIP event pair around every launch on
        its stream; returns the mean device time (ms) per launch name."""
        keep = self.cols, self.labels
        self._timing = []
        try:
            for i in range(n):
                cols, labels = batches[i % len(batches)]
                self.cols, self.labels = list(cols), labels.to(torch.int32)
                self._timing.append({})
                self.step()
            torch.cuda.synchronize(self.device)
            acc = {}
            for m in self._timing:
                for name, (a, b) in m.items():
                    acc.setdefault(name, []).append(a.elapsed_time(b))
        finally:
            self._timing = None
            self.cols, self.labels = keep
        return {k: sum(v) / len(v) for k, v in acc.items()}

    def capture_pool(self, batches: Sequence, steps_per_graph: int = 1, keep_graph: bool = False) -> None:
        """Graphs over resident input batches ((cols, labels) device tensors), read in place so a
        replay needs no input copy. Graph j runs full steps on batches j*k .. j*k+k-1 (k =
        ``steps_per_graph``, len(batches) % k == 0): k > 1 amortises the host cost of a graph
        launch over k steps."""
        k = int(steps_per_graph)
        if k < 1 or len(batches) % k:
            raise _lib.TTError("capture_pool: the batch count must be a multiple of steps_per_graph")
        staged = []
        for cols, labels in batches:
            for c in cols:
                if c.dtype != self.id_dtype or not c.is_contiguous() or c.numel() != self.B:
                    raise _lib.TTError("capture_pool: batch columns must match the step's id dtype and batch")
            staged.append((list(cols), labels.to(torch.int32).contiguous()))
        self._pool_inputs = getattr(self, "_pool_inputs", []) + [staged]  # alive as long as any graph
        self._prefault_due = True  # the next replay walks the tables' pages first (TableSet.prefault)
        self.pool_graphs = []
        for j in range(0, len(staged), k):
            self.capture(staged[j:j + k], keep_graph=keep_graph)
            self.pool_graphs.append(self.graph)
        self.steps_per_graph = k
