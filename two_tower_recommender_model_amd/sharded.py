"""The two-tower training step sharded over W MI355X (one process per GPU), single-hot features.

Semantics = DistributedModelParallel(TwoTowerTrainTask) + TrainPipelineSparseDist.progress of the
reference (03_model_training.py:798-829, :618): every table row-wise (block ceil(N/W)) or
table-wise sharded over the ranks, the towers data-parallel (DDP: gradients averaged over ranks),
each rank training on its own local batch of B pairs.

Pipelined schedule: TWO collectives per step, the route of every batch computed two steps ahead
(it depends only on that batch's ids). Per rank, step i (batch i's rows already returned, batch
i+1's keys already placed in exchange A's key region):

  T1 (indexed)    towers fwd/bwd reading rows_in[pos_in], dX -> exchange A's gradient region
  all-to-all A    [gradient rows(i) | keys(i+1)]                          requester -> owner
  launch U        owner's fused row-wise Adagrad(i) over the received gradient rows  |  T2(i):
                  the towers' weight gradients  |  count pass of route(i+2)
  launch G        owner's gather(i+1): the rows the received keys name (bf16) into exchange B,
                  filed for Adagrad(i+1)  |  the reduced tower gradient(i) x 1/W into the tower
                  block of every destination of exchange B  |  place pass of route(i+2) (ids %
                  N and drop-0 inline, segment (d, f) of fixed capacity) -> exchange A's key region
  all-to-all B    [rows(i+1) | tower gradient(i)]                         owner -> requester
  Adam(i)         fixed-order sum of the W received tower gradients (= DDP's mean all-reduce)

The tower weight gradients run beside the embedding update (launch U) and their reduction beside
the gather (launch G): T1, the two exchanges, U, G and Adam are the step's critical path. Every
exchange has a fixed size (per-destination capacities), so with RCCL (backend "nccl") the step is
captured into HIP graphs like the single-GPU step. Batch i+1's rows are gathered after Adagrad(i)
has updated the owner's shard, so results are those of the synchronous loop. The
embedding gradient a row receives is the sum over ranks of the per-rank mean-loss gradients
(TorchRec's sharded EBC semantics); lookups of a row are summed in ascending (source rank, slot)
order. ``step()`` (no next batch known) runs the same kernels in order with four exchanges.
A segment over capacity or a key outside a shard raises on ``check()`` (sticky device flags,
all-reduced over the ranks).
"""
from __future__ import annotations

import ctypes as C
import os
import threading
import time
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import _lib, ops
from ._lib import FeatureMeta, ShardSeg, check, id_dtype_code, ptr, ptr_array, stream_handle


# ---- collectives --------------------------------------------------------------------------------


class _Done:
    def wait(self):
        return None

    def is_completed(self):
        return True


def graph_safe_nccl_env() -> None:
    """Environment for a "nccl" (RCCL) process group whose collectives are captured into HIP graphs;
    call BEFORE dist.init_process_group. ProcessGroupNCCL's watchdog queries the end event of every
    eager work it tracks; with its CUDA-event cache on, a finished work's event goes back to the
    cache and is re-recorded by a collective issued during a later capture, and the watchdog's
    query of the old work then fails with hipErrorCapturedEvent (seen on MI355X: the process
    aborted at exit after a graphed run). With the cache off every work owns its event. Eager works
    are also retired before any capture (``TorchComm.retire``)."""
    import os

    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")


def _wait_for_watchdog(pg) -> None:
    """ProcessGroupNCCL::waitForPendingWorks through torch's private binding
    (``ProcessGroup._wait_for_pending_works``, present in torch 2.1 .. 2.10). Without it a capture
    after eager collectives can race the watchdog thread (``TorchComm.retire``), so its absence is an
    error, not a silent skip: graph capture is refused and ``capture_pool_or_eager`` / the drop-in
    fall back to eager steps."""
    fn = getattr(pg, "_wait_for_pending_works", None)
    if fn is None:
        raise _lib.TTError(f"torch {torch.__version__}: ProcessGroup._wait_for_pending_works is missing; RCCL "
                           "collectives cannot be captured safely (eager steps instead)")
    fn()


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
        self._eager: List = []

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits: Optional[List[int]] = None,
                   in_splits: Optional[List[int]] = None):
        """All-to-all along dim 0 (equal blocks, or the given fixed split sizes)."""
        if self.world == 1 and not self.always:
            out.copy_(inp)
            return
        capturing = torch.cuda.is_current_stream_capturing()
        w = dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits,
                                   group=self.group, async_op=not capturing)
        if w is not None:
            w.wait()  # the current stream waits for RCCL's; the handle is kept for retire()
            if len(self._eager) >= 64:
                self._eager = [h for h in self._eager if not h.is_completed()]
            self._eager.append(w)

    def retire(self, timeout_s: float = 60.0) -> None:
        """Wait until every eager collective issued so far is complete (device and watchdog view)
        — call before capturing collectives into a HIP graph."""
        torch.cuda.synchronize()
        t0 = time.monotonic()
        for w in self._eager:
            w.wait()
            while not w.is_completed():
                if time.monotonic() - t0 > timeout_s:
                    raise _lib.TTError("an eager collective did not complete before graph capture")
                time.sleep(0.001)
        self._eager.clear()
        # ProcessGroupNCCL's watchdog thread keeps a copy of every eager work (these and the untracked
        # synchronous ones: capacity / flag all-reduces) until a pass of its loop finds it complete,
        # queries its end event and erases it, destroying the event when it holds the last reference.
        # That thread runs in HIP's default (global) capture mode, so a query or destroy it makes
        # while this thread captures invalidates the capture (seen on MI355X once in ~10 runs:
        # hipErrorStreamCaptureInvalidated, then the watchdog aborting the process). Every eager work
        # is complete on the device now; ProcessGroupNCCL::waitForPendingWorks returns once the
        # watchdog's list is empty (it checks under the lock the watchdog holds for its whole pass),
        # after which the watchdog makes no HIP call until a new eager work exists, and captured
        # collectives are never handed to it.
        pg = self.group if self.group is not None else dist.distributed_c10d._get_default_group()
        if dist.get_backend(pg) == "nccl":
            _wait_for_watchdog(pg)

    def all_reduce_max_(self, t: torch.Tensor) -> None:
        if self.world > 1 or self.always:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)

    def gather_rows(self, local: torch.Tensor, spans: Sequence[Tuple[int, int]], full_rows: int):
        """Rank 0 receives every rank's row block (spans[r] = (first row, rows)) into one
        [full_rows, *] tensor (returned on rank 0, None elsewhere); point-to-point, so no rank
        ever holds more than its own shard plus, on rank 0, the result."""
        shape = tuple(local.shape[1:])
        if self.rank == 0:
            full = torch.empty((full_rows,) + shape, dtype=local.dtype, device=local.device)
            lo, n = spans[0]
            full[lo:lo + n].copy_(local[:n])
            for r in range(1, self.world):
                lo, n = spans[r]
                if n:
                    buf = torch.empty((n,) + shape, dtype=local.dtype, device=local.device)
                    dist.recv(buf, src=r, group=self.group)
                    full[lo:lo + n].copy_(buf)
            return full
        lo, n = spans[self.rank]
        if n:
            dist.send(local[:n].contiguous(), dst=0, group=self.group)
        return None

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> None:
        if self.world > 1:
            dist.broadcast(t, src=src, group=self.group)

    def recv_buffer(self, shape, dtype: torch.dtype, device) -> torch.Tensor:
        """A receive buffer of an all-to-all (zeroed)."""
        return torch.zeros(shape, dtype=dtype, device=device)


class _DeviceArray:
    """A device allocation as __cuda_array_interface__ (bytes), for torch.as_tensor."""

    def __init__(self, p: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (p, False), "version": 2}


class PeerComm(TorchComm):
    """TorchComm whose all-to-alls on the step's data path are device-initiated (the
    sharded steps' default at N > 1 through ``exchange_comm``, which runs ``self_test`` first and falls
    back to RCCL on every rank when it fails): every rank stores its blocks straight into the peers'
    receive buffers — allocated here (``recv_buffer``, fine-grained device memory) and mapped into
    every other rank's process with hipIpcOpenMemHandle — and signals a flag word per (peer, source);
    the receiver's wait kernel spins on its W words (csrc/peer.hip: a put kernel, then one wave that
    signals and waits). No RCCL kernel runs on the step path, and the exchange is capturable whatever
    the process group's backend (gloo included: it only carries the setup). The other collectives
    (capacities, flags, checkpoints) stay torch.distributed. A wait past ``timeout_s`` gives up and
    sets a sticky error word that ``check()`` of the step raises on: the results of every step from
    then on are invalid and the run must be restarted (nothing clears the word). Replaces the
    all_to_all_single calls TorchComm issues (TorchRec's input_dist / output_dist all-to-alls and DDP's
    tower all-reduce under DistributedModelParallel, 03_model_training.py:812-815).

    Verified here: ranks sharing one GPU (world 1, and W processes on the test box's one MI355X),
    with both signalling scopes (``TT_PEER_SYSTEM_SCOPE=1`` forces the cross-device one). Ranks on
    different GPUs (xGMI) run the same protocol at system scope; only the startup self-test checks it
    on that hardware."""

    def __init__(self, group=None, timeout_s: float = 60.0, device=None, memory: Optional[str] = None):
        """memory: None (fine-grained, or torch's allocator when every rank is on one device and the
        fine-grained allocation is refused), "fine-grained" (hipDeviceMallocFinegrained, coherent
        across devices; required for ranks on different devices) or "device" (torch's allocator:
        coarse-grained, coherent only within one device: refused for ranks on different devices).
        timeout_s: how long a wait kernel spins for a peer's signal before it gives up (the
        process-group timeout's order: a rank may lag by a graph capture or a slow first batch)."""
        super().__init__(group, always_collective=True)
        if self.world > _lib.TT_PEER_MAXW:
            raise _lib.TTError(f"PeerComm: at most {_lib.TT_PEER_MAXW} ranks")
        self.timeout_s = float(timeout_s)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.memory = memory or os.environ.get("TT_PEER_MEMORY") or None
        if self.memory not in (None, "fine-grained", "device"):
            raise _lib.TTError('PeerComm: memory is "fine-grained" or "device"')
        self._bufs: Dict[int, dict] = {}
        self._own: List[int] = []
        self._imports: Dict[bytes, int] = {}
        self._puts: Dict[tuple, _lib.PeerPut] = {}
        # every rank on this one device (world 1, or ranks sharing a GPU): agent-scope signals suffice
        ident = self._device_identity()
        idents = [None] * self.world
        if self.world > 1:
            dist.all_gather_object(idents, ident, group=self.group)
        else:
            idents[0] = ident
        self.same_device = ident is not None and all(i == ident for i in idents)
        self.shared_gpu = self.same_device  # the truth, whatever scope the signalling is forced to
        if os.environ.get("TT_PEER_SYSTEM_SCOPE") == "1":  # tests / measurement: the multi-device signalling
            self.same_device = False
        if self.memory == "device" and not self.same_device:
            raise _lib.TTError('PeerComm: memory="device" (coarse-grained) is coherent within one device only; '
                               "ranks on different devices need fine-grained memory")

    def _device_identity(self):
        p = torch.cuda.get_device_properties(self.device)
        ident = tuple(str(getattr(p, a, "")) for a in ("uuid", "pci_domain_id", "pci_bus_id", "pci_device_id"))
        return ident if any(ident) else None  # unknown: treated as different devices (system scope)

    def _alloc(self, nbytes: int) -> torch.Tensor:
        """Fine-grained device memory (setup only: tt_peer_alloc allocates and synchronises). Torch's
        coarse-grained allocator only when asked for, or when every rank is on this one device and
        the fine-grained allocation was refused (coherent there: the kernel boundaries publish it)."""
        lib = _lib.load()
        if self.memory in (None, "fine-grained"):
            p = C.c_void_p()
            rc = lib.tt_peer_alloc(nbytes, C.byref(p))
            if rc == 0:
                try:
                    raw = torch.as_tensor(_DeviceArray(p.value, nbytes), device=self.device)
                except Exception as e:  # noqa: BLE001
                    check(lib.tt_peer_free(p), "peer_free")
                    if self.memory == "fine-grained" or not self.same_device:
                        raise _lib.TTError(f"PeerComm: torch cannot wrap the fine-grained allocation ({e})") from e
                else:
                    self._own.append(p.value)
                    self.memory = "fine-grained"
                    return raw
            elif self.memory == "fine-grained" or not self.same_device:
                check(rc, "peer_alloc")
        self.memory = "device"
        return torch.zeros(nbytes, dtype=torch.uint8, device=self.device)

    def _agree(self, ok: bool) -> bool:
        """Collective: True iff ``ok`` on every rank."""
        t = torch.tensor([0 if ok else 1], dtype=torch.int32, device=self.device)
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item()) == 0

    def recv_buffer(self, shape, dtype: torch.dtype, device) -> torch.Tensor:
        """Collective (every rank, same order): a zeroed receive buffer followed by this exchange's W
        flag words, exported to every other rank; the peers' buffers are mapped in return. Setup
        only (allocates, synchronises). A local failure (allocation, export, import) is agreed on
        before anyone raises, so every rank raises the same error and none waits in a collective."""
        lib = _lib.load()
        shape = tuple(int(s) for s in (shape if isinstance(shape, (tuple, list)) else (shape,)))
        n = 1
        for s in shape:
            n *= s
        item = torch.empty((), dtype=dtype).element_size()
        body = -(-max(1, n * item) // 256) * 256
        why = ""
        raw, mine = None, None
        try:
            raw = self._alloc(body + 256)
            h = (C.c_char * _lib.TT_PEER_HANDLE_BYTES)()
            off = C.c_int64()
            if self.world > 1:
                check(lib.tt_peer_export(C.c_void_p(raw.data_ptr()), h, C.byref(off)), "peer_export")
            mine = (bytes(h), int(off.value), body)
        except Exception as e:  # noqa: BLE001 - agreed on below
            why = f"rank {self.rank}: {e}"
        allv = [None] * self.world
        if self.world > 1:
            dist.all_gather_object(allv, mine, group=self.group)
        else:
            allv[0] = mine
        peers = []
        if all(v is not None for v in allv):
            try:
                for s, (hs, o, b) in enumerate(allv):
                    if s == self.rank:
                        peers.append((raw.data_ptr(), b))
                        continue
                    if hs not in self._imports:
                        p = C.c_void_p()
                        check(lib.tt_peer_import(hs, C.byref(p)), "peer_import")
                        self._imports[hs] = p.value
                    peers.append((self._imports[hs] + o, b))
            except Exception as e:  # noqa: BLE001
                why = why or f"rank {self.rank}: {e}"
        elif not why:
            why = "a peer could not allocate or export its buffer"
        if not self._agree(not why):
            raise _lib.TTError(f"PeerComm.recv_buffer failed on some rank{': ' + why if why else ''}")
        buf = raw[:n * item].view(dtype).view(shape)
        self._bufs[buf.data_ptr()] = {"peers": peers, "flags": raw[body:body + 4 * self.world].view(torch.int32),
                                      "state": torch.zeros(1, dtype=torch.int32, device=self.device),
                                      "raw": raw, "body": body}
        return buf

    def self_test(self, nbytes: int = 1 << 16, rounds: int = 3, timeout_s: float = 10.0) -> Tuple[bool, str]:
        """Collective startup check of the protocol on this node: ``rounds`` all-to-alls of a
        (source, destination, round)-tagged pattern through one receive buffer, at the signalling
        scope the steps will use, each checked on the host; the wait kernels give up after
        ``timeout_s``. Returns (ok on every rank, the first reason a rank gave)."""
        why = ""
        W, r = self.world, self.rank
        n = max(64, nbytes // 4 // 64 * 64)  # int32 per block
        keep, self.timeout_s = self.timeout_s, min(self.timeout_s, float(timeout_s))
        try:
            out = self.recv_buffer((W * n,), torch.int32, self.device)
            idx = torch.arange(n, dtype=torch.int64, device=self.device)
            for k in range(rounds):
                inp = torch.cat([((r * 1_000_003 + d * 7_919 + k * 104_729 + idx * 31) % 2_000_000_011).to(torch.int32)
                                 for d in range(W)])
                self.all_to_all(out, inp)
                torch.cuda.synchronize(self.device)
                if int(self.err.item()):
                    why = f"rank {r}: a wait timed out ({timeout_s} s) in round {k}"
                else:
                    want = torch.cat([((s * 1_000_003 + r * 7_919 + k * 104_729 + idx * 31) % 2_000_000_011)
                                      .to(torch.int32) for s in range(W)])
                    if not torch.equal(out, want):
                        why = f"rank {r}: round {k}: {int((out != want).sum())} of {W * n} received words differ"
                # every rank checks before anyone overwrites the buffer; all stop together
                if not self._agree(not why):
                    break
        except Exception as e:  # noqa: BLE001 - a local error (setup is agreed on inside recv_buffer)
            why = why or f"rank {r}: {e}"
            self._agree(False)
        finally:
            self.timeout_s = keep
        ok = self._agree(not why)  # every path above ran the same collectives on every rank
        if not ok and not why:
            why = "a peer failed its check"
        return ok, why

    supports_direct = True

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits: Optional[List[int]] = None,
                   in_splits: Optional[List[int]] = None, stored: bool = False):
        """All-to-all along dim 0 into a buffer from ``recv_buffer``: block d of ``inp`` (``in_splits[d]``
        rows, or equal blocks) lands in rank d's buffer at block ``rank``; every rank's blocks are
        equal-sized at the receiver (what the sharded step's fixed layout guarantees). ``stored``:
        the producers already stored every block at its destination (``direct``): only the signal /
        wait runs."""
        e = self._bufs.get(out.data_ptr())
        if e is None:
            raise _lib.TTError("PeerComm.all_to_all: the receive buffer was not allocated by recv_buffer()")
        W, r = self.world, self.rank
        key = (out.data_ptr(), inp.data_ptr(), tuple(in_splits or ()), inp.shape[0], bool(stored))
        put = self._puts.get(key)
        if put is None:
            rowb = inp.element_size() * (inp.numel() // max(1, inp.shape[0]))
            sizes = list(in_splits) if in_splits is not None else [inp.shape[0] // W] * W
            if len(sizes) != W or sum(sizes) > inp.shape[0]:
                raise _lib.TTError("PeerComm.all_to_all: one block per rank within the input")
            mine = (out_splits[0] if out_splits is not None else out.shape[0] // W) * rowb
            if out_splits is not None and any(s != out_splits[0] for s in out_splits):
                raise _lib.TTError("PeerComm.all_to_all: equal receive blocks only")
            if mine * W > out.numel() * out.element_size() or sizes[r] * rowb != mine:
                raise _lib.TTError("PeerComm.all_to_all: receive blocks do not match the senders' blocks")
            put = _lib.PeerPut()
            put.W, put.rank, put.src, put.state = W, r, inp.data_ptr(), e["state"].data_ptr()
            put.same_device = 1 if self.same_device else 0
            o = 0
            for d in range(W):
                base, body = e["peers"][d]
                put.src_off[d] = o * rowb
                put.len[d] = 0 if stored else sizes[d] * rowb
                put.dst[d] = base + r * sizes[d] * rowb
                put.flag[d] = base + body + 4 * r
                o += sizes[d]
            self._puts[key] = put
        check(_lib.load().tt_peer_exchange(C.byref(put), e["flags"].data_ptr(), self.err.data_ptr(), self.timeout_s,
                                           stream_handle(out.device)), "peer_exchange")

    def block_dst(self, out: torch.Tensor, inp: torch.Tensor, out_splits: Optional[List[int]] = None,
                  in_splits: Optional[List[int]] = None) -> List[Tuple[int, int, int]]:
        """Per destination d of ``all_to_all(out, inp, ...)``: (byte offset of block d in ``inp``,
        its bytes, the mapped address where it lands at d)."""
        e = self._bufs.get(out.data_ptr())
        if e is None:
            raise _lib.TTError("PeerComm.block_dst: the receive buffer was not allocated by recv_buffer()")
        W, r = self.world, self.rank
        rowb = inp.element_size() * (inp.numel() // max(1, inp.shape[0]))
        sizes = list(in_splits) if in_splits is not None else [inp.shape[0] // W] * W
        out_rows = out_splits[0] if out_splits is not None else out.shape[0] // W
        if len(sizes) != W or sizes[r] != out_rows:
            raise _lib.TTError("PeerComm.block_dst: receive blocks do not match the senders' blocks")
        res, o = [], 0
        for d in range(W):
            res.append((o * rowb, sizes[d] * rowb, e["peers"][d][0] + r * sizes[d] * rowb))
            o += sizes[d]
        return res

    def direct(self, out: torch.Tensor, inp: torch.Tensor, unit_bytes: int, out_splits: Optional[List[int]] = None,
               in_splits: Optional[List[int]] = None, copy: Optional[Sequence[Tuple[int, int]]] = None,
               epoch: bool = False):
        """tt_peer_direct_t for a producer of ``inp`` (units of ``unit_bytes``, counted from ``inp``'s
        start) whose all-to-all into ``out`` then runs with ``stored=True``: block d's units go to
        their place in rank d's receive buffer. ``copy[d] = (lo, hi)``: bytes [lo, hi) of block d
        (relative to its start) that the producer copies to rank d beside its units. ``epoch``: the
        producer advances the exchange's epoch, and its consumer signals / waits in-launch
        (``wait_desc``) instead of the all-to-all call."""
        blocks = self.block_dst(out, inp, out_splits, in_splits)
        x = _lib.PeerDirect()
        x.W = self.world
        if epoch:
            x.epoch = self._bufs[out.data_ptr()]["state"].data_ptr()
        for d, (off, n, dst) in enumerate(blocks):
            if off % unit_bytes:
                raise _lib.TTError("PeerComm.direct: a block does not start on a unit")
            x.first_row[d] = off // unit_bytes
            x.row0[d] = dst
            if copy is not None:
                lo, hi = copy[d]
                if not 0 <= lo <= hi <= n or (lo | hi | off | dst | inp.data_ptr()) % 16:
                    raise _lib.TTError("PeerComm.direct: copy ranges must be 16-B aligned inside the block")
                x.copy_src[d] = inp.data_ptr() + off + lo
                x.copy_dst[d] = dst + lo
                x.copy_len[d] = hi - lo
        return x

    @property
    def in_launch_wait(self) -> bool:
        """Whether a consumer launch may signal / wait in-launch (tt_peer_wait_t): ranks on different
        devices or one rank. Ranks sharing a device are excluded: one rank's spinning workgroups
        could hold every CU while a peer's producer waits for one."""
        return self.world == 1 or not self.shared_gpu

    def wait_desc(self, out: torch.Tensor):
        """tt_peer_wait_t of the exchange into ``out`` (a buffer from recv_buffer) for a consumer
        launch that signals / waits in-launch; its producer took ``direct(..., epoch=True)``."""
        e = self._bufs.get(out.data_ptr())
        if e is None:
            raise _lib.TTError("PeerComm.wait_desc: the receive buffer was not allocated by recv_buffer()")
        if not self.in_launch_wait:
            raise _lib.TTError("PeerComm.wait_desc: ranks share a device (use the all-to-all's signal / wait)")
        w = _lib.PeerWait()
        w.W, w.sys = self.world, 0 if self.same_device else 1
        for d in range(self.world):
            base, body = e["peers"][d]
            w.flag[d] = base + body + 4 * self.rank
        w.flags, w.epoch, w.err = e["flags"].data_ptr(), e["state"].data_ptr(), self.err.data_ptr()
        w.timeout_ticks = int(min(self.timeout_s * 1e8, 9e17))  # s_memrealtime: 100 MHz
        return w

    def close(self) -> None:
        """Unmap the peers' buffers and free this rank's (the buffers from recv_buffer are invalid after)."""
        torch.cuda.synchronize(self.device)
        lib = _lib.load()
        for p in self._imports.values():
            check(lib.tt_peer_unimport(C.c_void_p(p)), "peer_unimport")
        self._imports.clear()
        self._bufs.clear()
        self._puts.clear()
        for p in self._own:
            check(lib.tt_peer_free(C.c_void_p(p)), "peer_free")
        self._own.clear()


def _probe_exchanges(pc: "PeerComm", group, device, block_bytes: Sequence[int], iters: int = 10):
    """Collective: the mean time (ms) of one round of all-to-alls with destination blocks of
    ``block_bytes`` each, through ``pc`` and through RCCL (all_to_all_single), max over the ranks."""
    tc = TorchComm(group, always_collective=True)
    W = pc.world
    res = []
    for comm in (pc, tc):
        tot = 0.0
        for nb in block_bytes:
            n = max(64, int(nb) // 4 // 64 * 64)  # int32 words per destination block
            inp = torch.zeros(W * n, dtype=torch.int32, device=device)
            out = (pc.recv_buffer((W * n,), torch.int32, device) if comm is pc
                   else torch.empty(W * n, dtype=torch.int32, device=device))
            for _ in range(3):
                comm.all_to_all(out, inp)
            torch.cuda.synchronize(device)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                comm.all_to_all(out, inp)
            e1.record()
            torch.cuda.synchronize(device)
            tot += e0.elapsed_time(e1) / iters
        res.append(tot)
    tc.retire()
    # a timed-out wait on any rank (sticky err) makes every rank read the peer exchange as unusable
    late = int(pc.err.item()) != 0
    t = torch.tensor(res + [1.0 if late else 0.0], dtype=torch.float64, device=device)
    if W > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    if float(t[2]) > 0:
        return float("inf"), float(t[1])
    return float(t[0]), float(t[1])


def exchange_comm(kind: str = "auto", group=None, device=None, verbose: bool = True,
                  probe: Optional[Sequence[int]] = None):
    """The sharded steps' comm (collective: every rank calls it with the same ``kind``).
    "rccl": TorchComm (all_to_all_single, RCCL over xGMI with backend "nccl"); "peer": PeerComm, the
    device-initiated exchange, after its startup ``self_test`` — raises if the test fails; "auto"
    (the default): PeerComm when its self-test passes on every rank, else TorchComm on every rank
    (the reason printed on rank 0). ``probe`` (auto, backend "nccl"): the step's per-destination
    block bytes; after the self-test both exchanges are timed on them (eager, max over ranks) and
    RCCL is taken if the device-initiated one is more than 10 % slower — a guard for interconnects
    where its stores do not pay. Returns (comm, description)."""
    if kind not in ("auto", "peer", "rccl"):
        raise _lib.TTError(f"exchange_comm: kind is auto, peer or rccl, got {kind!r}")
    if kind == "rccl":
        return TorchComm(group, always_collective=True), "RCCL all_to_all_single"
    why = ""
    try:
        pc = PeerComm(group, device=device)
    except _lib.TTError as e:  # raised on every rank alike (argument / memory-kind checks)
        pc, why = None, str(e)
    if pc is not None:
        ok, why = pc.self_test()
        if ok and kind == "auto" and probe and dist.get_backend(group) == "nccl":
            tp, tr = _probe_exchanges(pc, group, device, probe)
            timing = f"probe {tp * 1e3:.1f} us against RCCL {tr * 1e3:.1f} us"
            if tp > 1.1 * tr:
                pc.close()
                if verbose and dist.get_rank(group) == 0:
                    import sys

                    print(f"exchange_comm: device-initiated exchange slower ({timing}); RCCL all-to-alls",
                          file=sys.stderr)
                return TorchComm(group, always_collective=True), f"RCCL all_to_all_single (peer {timing})"
            return pc, (f"device-initiated puts into IPC-mapped peer buffers ({pc.memory} memory, self-test "
                        f"passed, {timing})")
        if ok:
            return pc, f"device-initiated puts into IPC-mapped peer buffers ({pc.memory} memory, self-test passed)"
        pc.close()
    if kind == "peer":
        raise _lib.TTError(f"PeerComm self-test failed: {why}")
    if verbose and dist.get_rank(group) == 0:
        import sys

        print(f"exchange_comm: device-initiated exchange unavailable ({why}); RCCL all-to-alls", file=sys.stderr)
    return TorchComm(group, always_collective=True), f"RCCL all_to_all_single (peer self-test failed: {why})"


class ThreadComm:
    """W ranks as W threads of ONE process on one device (tests): each collective is a rendezvous
    on a barrier; all-to-all copies the peers' blocks."""

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

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits: Optional[List[int]] = None,
                   in_splits: Optional[List[int]] = None):
        W = self.world
        self._exchange((inp, in_splits))
        o = 0
        for s in range(W):
            src, splits = self.shared.slots[s]
            if splits is None:
                n = src.shape[0] // W
                lo, hi = self.rank * n, (self.rank + 1) * n
            else:
                lo = sum(splits[:self.rank])
                hi = lo + splits[self.rank]
            out[o:o + hi - lo].copy_(src[lo:hi])
            o += hi - lo
        torch.cuda.current_stream().synchronize()
        self.shared.barrier.wait()

    def retire(self, timeout_s: float = 60.0) -> None:
        torch.cuda.synchronize()

    def all_reduce_max_(self, t: torch.Tensor) -> None:
        self._exchange(t.clone())
        acc = self.shared.slots[0]
        for s in range(1, self.world):
            acc = torch.maximum(acc, self.shared.slots[s])
        torch.cuda.current_stream().synchronize()
        self.shared.barrier.wait()
        t.copy_(acc)

    def gather_rows(self, local: torch.Tensor, spans: Sequence[Tuple[int, int]], full_rows: int):
        self._exchange(local)
        full = None
        if self.rank == 0:
            full = torch.empty((full_rows,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
            for r in range(self.world):
                lo, n = spans[r]
                full[lo:lo + n].copy_(self.shared.slots[r][:n])
        torch.cuda.current_stream().synchronize()
        self.shared.barrier.wait()
        return full

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> None:
        self._exchange(t.clone())
        v = self.shared.slots[src]
        torch.cuda.current_stream().synchronize()
        self.shared.barrier.wait()
        t.copy_(v)

    def recv_buffer(self, shape, dtype: torch.dtype, device) -> torch.Tensor:
        return torch.zeros(shape, dtype=dtype, device=device)


# ---- the step -----------------------------------------------------------------------------------


def default_capacity(B: int, W: int, factor: float = 1.25) -> int:
    """Per-(owner, feature) segment capacity of a row-wise feature: the expected B/W lookups per
    owner with slack for the binomial spread of uniformly spread ids (B/W + 6 sigma at B = 8192,
    W = 8 is ~1200)."""
    if W == 1:
        return B
    c = int(factor * B / W) + 64
    return min(B, (c + 7) // 8 * 8)


def segment_counts(cols: Sequence[torch.Tensor], num_embeddings: Sequence[int], block_sizes: Sequence[int],
                   owners: Sequence[int], W: int) -> torch.Tensor:
    """[W, F] kept lookups per (owner, feature) of one batch (host check of a capacity)."""
    out = torch.zeros(W, len(cols), dtype=torch.int64)
    for f, c in enumerate(cols):
        c = c.to(torch.int64)
        row = torch.remainder(c[c != 0], int(num_embeddings[f]))
        d = row // block_sizes[f] if block_sizes[f] > 0 else torch.full_like(row, int(owners[f]))
        out[:, f] = torch.bincount(d.cpu(), minlength=W)[:W]
    return out


class FusedShardedTwoTowerStep:
    def __init__(self, comm, num_embeddings: Sequence[int], embedding_dim: int, layer_sizes: Sequence[int],
                 batch_size: int, device: torch.device, sharding: Optional[Sequence[str]] = None,
                 tw_owners: Optional[Sequence[int]] = None, lr_emb: float = 0.01, lr_dense: float = 0.01,
                 eps: float = 1e-10, id_dtype: torch.dtype = torch.int64, seed: int = 0,
                 capacity=None, full_tables: Optional[Sequence[torch.Tensor]] = None,
                 num_query_features: Optional[int] = None, overlap: bool = False,
                 tables: Optional[ops.TableSet] = None):
        """Single-hot features, one table each: features 0 .. Fq-1 feed the query tower (their rows
        concatenated in that order: torch.cat([kt[f] for f in query features]),
        03_model_training.py:420-425), features Fq .. F-1 the candidate tower; ``num_query_features``
        = Fq (default 1 with two features: the reference's user / item towers). ``sharding[f]`` is
        "row_wise" (default) or "table_wise" (owner ``tw_owners[f]``). ``capacity``: slots per
        (owner, row-wise feature) segment — an int, a per-feature list, or None (default_capacity);
        a table-wise feature's owner segment holds B. ``full_tables`` (CPU, optional) give the
        initial weights; otherwise each rank draws its shard from U(-sqrt(1/N), sqrt(1/N)) (torchrec
        EBC init). Tower parameters are initialised from ``seed`` identically on every rank (what
        DDP's initial broadcast guarantees). Two features run T1 in its fused 2-layer form
        (tt_tower_fwd_bwd_indexed2_bf16); more features per tower (BASELINE configs 3 and 4) run the
        general T1 over the concatenated rows (tt_tower_fwd_bwd_indexed_multi_bf16). ``overlap``: the
        pipelined step runs the towers' weight gradients (T2) on a parallel stream beside exchange A
        and the owner's update (else inside launch U, one stream; the default: the parallel branch
        measured 94.1 against 70.5 us per world-1 step, profiles/r03_bench_sharded_w1*.log).
        ``tables``: adopt this rank's shards instead of allocating them — table f of the TableSet is
        feature f's local shard (rows [row_lo, row_lo + local rows) of a row-wise table, the whole
        table-wise table on its owner, 0 rows elsewhere; ops.TableSet.view_of over a
        ShardedEmbeddingBagCollection's storage, dropin.py): trained in place, not initialised."""
        self.comm = comm
        self.W, self.rank = comm.world, comm.rank
        self.device = torch.device(device)
        dev = self.device
        self.F = len(num_embeddings)
        if self.F < 2 or self.F > _lib.TT_MAX_FEATURES:
            raise _lib.TTError("sharded step: 2..64 features")
        self.Fq = int(num_query_features) if num_query_features is not None else (1 if self.F == 2 else 0)
        if not 1 <= self.Fq < self.F:
            raise _lib.TTError("sharded step: num_query_features must leave both towers at least one feature")
        self.multi = not (self.F == 2 and self.Fq == 1)
        self.B = int(batch_size)
        self.D = int(embedding_dim)
        self.N = [int(n) for n in num_embeddings]
        self.layer_sizes = [int(x) for x in layer_sizes]
        self.lr_emb, self.lr_dense, self.eps = float(lr_emb), float(lr_dense), float(eps)
        self.id_dtype = id_dtype
        sharding = list(sharding or ["row_wise"] * self.F)
        tw_owners = list(tw_owners or [f % self.W for f in range(self.F)])
        if len(sharding) != self.F or len(tw_owners) != self.F:
            raise _lib.TTError("sharded step: one sharding / owner per feature")
        self.sharding = sharding
        W, r, F, B, D = self.W, self.rank, self.F, self.B, self.D
        if D % 4 or D > 128 or (self.multi and (D % 16 or 128 % D)):
            raise _lib.TTError("sharded step: D % 4 == 0 and D <= 128 (several features per tower: D in 16, 32, "
                               "64, 128)")
        self.in_dims = [self.Fq * D, (F - self.Fq) * D]
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
        self._adopted = tables is not None
        if self._adopted:
            # a shard of no rows may be a one-row placeholder (ShardedEmbeddingBagCollection allocates
            # max(1, n) rows, torchrec/distributed/embeddingbag.py): no key ever reaches it
            if tables.T != F or tables.dims != [D] * F or tables.device != dev or \
                    any(tables.rows[f] != local_rows[f] and not (local_rows[f] == 0 and tables.rows[f] <= 1)
                        for f in range(F)):
                raise _lib.TTError(f"sharded step: adopted tables must be this rank's shards (rows {local_rows}, "
                                   f"dim {D}), feature f -> table f; got rows {tables.rows}")
            self.tables = tables
        else:
            self.tables = ops.TableSet([max(1, n) for n in local_rows], [D] * F, list(range(F)), dev)
            self.tables.weights.zero_()  # a feature this rank holds no rows of keeps one zero dummy row
        for f in range(F if not self._adopted else 0):
            view = self.tables.table_view(f)
            if local_rows[f] == 0:
                continue
            if full_tables is not None:
                if local_rows[f]:
                    lo = self.row_lo[f]
                    view[:local_rows[f]].copy_(full_tables[f][lo:lo + local_rows[f]])
            else:
                a = (1.0 / self.N[f]) ** 0.5
                view.uniform_(-a, a, generator=torch.Generator(device=dev).manual_seed(seed * 1000 + 17 * r + f))
        # ---- towers (data-parallel replicas)
        in_cols = [0, self.in_dims[0]]
        if not ops.FusedTowers.supported(self.in_dims, self.layer_sizes, in_cols, B) or \
                (not self.multi and len(self.layer_sizes) != 2):
            raise _lib.TTError("sharded step: unsupported tower shape (two features: 2 layers, fused T1; inputs up "
                               "to 1024 wide, widths 32..128)")
        self.towers = ops.FusedTowers(self.in_dims, self.layer_sizes, in_cols, B, dev,
                                      flags=_lib.TT_TOWER_GENERAL_T1 if self.multi else 0)
        P = self.towers.num_params
        self.params = torch.empty(P, dtype=torch.float32, device=dev)
        self.grads = torch.zeros(P, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(P, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(P, dtype=torch.float32, device=dev)
        self.adam_state = torch.zeros(2, dtype=torch.int64, device=dev)
        g = torch.Generator().manual_seed(seed + 1)
        chunks = []
        for t in range(2):
            i = self.in_dims[t]
            for out in self.layer_sizes:
                bound = 1.0 / i ** 0.5
                chunks += [torch.empty(out, i).uniform_(-bound, bound, generator=g).flatten(),
                           torch.empty(out).uniform_(-bound, bound, generator=g)]
                i = out
        self.params.copy_(torch.cat(chunks))
        self.towers.update(self.params, do_adam=False)
        # ---- exchange layout (fixed sizes, identical arithmetic on every rank)
        if capacity is None:
            caps_f = [default_capacity(B, W)] * F
        elif isinstance(capacity, (list, tuple)):
            caps_f = [int(c) for c in capacity]
        else:
            caps_f = [int(capacity)] * F
        self.caps_f = caps_f
        self.cap = [[(caps_f[f] if sharding[f] == "row_wise" else (B if self.owner[f] == d else 0))
                     for f in range(F)] for d in range(W)]
        self._layout()
        # ---- buffers
        self.sendA = torch.zeros(self.A_total, dtype=torch.float32, device=dev)
        # receive buffers from the comm when it provides them (PeerComm: mapped into every peer for
        # its device-initiated puts); plain device tensors for any other comm
        recv = getattr(comm, "recv_buffer", None) or (lambda shape, dtype, device: torch.zeros(shape, dtype=dtype,
                                                                                              device=device))
        self.recvA = recv((W * self.Asz[r],), torch.float32, dev)
        self.rows_out = torch.zeros(W * self.RSTR, D, dtype=torch.bfloat16, device=dev)
        self.rows_in = recv((W * self.RSTR, D), torch.bfloat16, dev)
        self.pos_in = torch.full((2, F * B), -1, dtype=torch.int32, device=dev)
        self.pos_out = torch.full((2, F * B), -1, dtype=torch.int32, device=dev)
        self.flags = torch.zeros(2, dtype=torch.int32, device=dev)  # {overflow, bad key}
        self.route_ws = torch.empty(_lib.load().tt_shard_route_workspace_bytes(F, B), dtype=torch.uint8, device=dev)
        segs = (ShardSeg * (W * F))()
        for d in range(W):
            for f in range(F):
                e = segs[d * F + f]
                ids64 = (self.A_off[d] + self.S[d] * D) // 2
                e.cap = self.cap[d][f]
                e.key_index = ids64 + F + self.seg_off[d][f]
                e.cnt_index = ids64 + f
                e.pos_in = self.RB_off[d] + self.seg_off[d][f]
                e.pos_out = self.A_off[d] // D + self.seg_off[d][f]
        raw = torch.frombuffer(bytearray(bytes(segs)), dtype=torch.uint8)
        self.segs = raw.to(dev)
        # dedup workspaces: batch i inserts at gather(i), Adagrad(i) consumes: two in flight
        self.max_lookups = max(1, W * self.S[r])
        nbytes = _lib.load().tt_dedup_workspace_bytes(self.max_lookups)
        self.dd_ws = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(2)]
        self._init_dedup()
        # Adagrad over the received gradient rows: one pseudo-feature per source block
        self._fm_src = (FeatureMeta * W)()
        for s in range(W):
            self._fm_src[s].table = 0
            self._fm_src[s].out_offset = 0
            self._fm_src[s].out_row = s * self.Asz[r] // D
        self._ne = (C.c_int64 * F)(*self.N)
        self._bs = (C.c_int64 * F)(*self.block)
        self._ow = (C.c_int32 * F)(*self.owner)
        self._segoff_me = (C.c_int64 * F)(*self.seg_off[r])
        # this rank's tower gradient x 1/W into exchange B's tower block of every destination (float
        # offsets into rows_out), and where Adam finds the W received ones in rows_in
        self._tw_off = (C.c_int64 * W)(*[(d * self.RSTR + self.Smax) * D // 2 for d in range(W)])
        self._tw_in = self.Smax * D // 2
        self._tw_stride = self.RSTR * D // 2
        # ---- step inputs / outputs
        self.cols = [torch.zeros(B, dtype=id_dtype, device=dev) for _ in range(F)]
        self.labels = torch.zeros(B, dtype=torch.int32, device=dev)
        self.logits = torch.empty(B, dtype=torch.float32, device=dev)
        self.loss = torch.zeros((), dtype=torch.float32, device=dev)
        # direct exchange (PeerComm, two features): T1 stores its gradient rows and copies the key
        # region straight into the owners' exchange-A buffers, launch G its gathered rows and the
        # tower gradient into the requesters' exchange-B buffers; the exchanges are then only their
        # signal / wait (TT_PEER_DIRECT=0: the put kernels instead)
        self.direct = (getattr(comm, "supports_direct", False) and not self.multi
                       and os.environ.get("TT_PEER_DIRECT", "1") != "0")
        # ... and, opt-in (TT_PEER_MERGED=1; ranks on different devices, or one rank), with in-launch
        # waits: no exchange kernel at all — launch U signals / waits exchange A, Adam exchange B.
        # Same-box A/B at world 1: 53.2 vs 52.6 us (agent scope), 53.3 vs 53.5 us (system scope)
        # against the signal / wait kernels (profiles/r06i_ab_in_launch_waits.log): not the default
        # until a multi-GPU run shows the overlap it buys there
        self.merged = (self.direct and getattr(comm, "in_launch_wait", False)
                       and os.environ.get("TT_PEER_MERGED", "0") == "1")
        if self.direct:
            self._dA = comm.direct(self.recvA, self.sendA, 4 * D, out_splits=[self.Asz[r]] * W,
                                   in_splits=list(self.Asz),
                                   copy=[(4 * self.S[d] * D, 4 * self.Asz[d]) for d in range(W)], epoch=self.merged)
            self._dB = comm.direct(self.rows_in, self.rows_out, 2 * D, out_splits=[self.RSTR] * W,
                                   in_splits=[self.RSTR] * W, epoch=self.merged)
            base = self.rows_out.data_ptr()
            offs = []
            for d in range(W):
                addr = self._dB.row0[d] + 2 * D * self.Smax  # the tower block of my block at rank d
                if (addr - base) % 4:
                    raise _lib.TTError("sharded step: exchange B's tower block is not 4-B aligned")
                offs.append((addr - base) // 4)
            self._tw_off_direct = (C.c_int64 * W)(*offs)
        if self.merged:
            self._wA = comm.wait_desc(self.recvA)
            self._wB = comm.wait_desc(self.rows_in)
        self.overlap = bool(overlap)
        self.side = torch.cuda.Stream(device=dev) if self.overlap else None
        self.pool_graphs: list = []
        self.small_graphs: list = []
        self.cursor = None  # pipelined pool: index of the batch whose rows are staged in rows_in
        torch.cuda.synchronize(dev)

    # ------------------------------------------------------------------------------------------
    def _init_dedup(self) -> None:
        for ws in self.dd_ws:
            check(_lib.load().tt_dedup_workspace_init(ptr(ws), ws.numel(), self.max_lookups,
                                                      stream_handle(self.device)), "dedup_workspace_init")

    def reset_pipeline(self) -> None:
        """Drop the pipelined state (the staged rows of the batch at the cursor and the keys both
        dedup tables hold for it and the next batch): the next pipelined run primes again. Needed
        whenever the staged state is stale or was never consumed: a capture that was refused after
        ``prime`` (its steps never ran), a ``load_state_dict`` in the middle of a run, a switch
        between the synchronous and the pipelined step. A dedup table filed twice with the same keys
        would join its own slots: those rows would never be updated."""
        torch.cuda.synchronize(self.device)
        self._init_dedup()
        self.cursor = None

    def _layout(self) -> None:
        W, F, D, P = self.W, self.F, self.D, self.towers.num_params
        rup = lambda x, m: -(-x // m) * m  # noqa: E731
        self.Ppad = rup(P, D)
        self.S = [sum(self.cap[d]) for d in range(W)]
        self.seg_off = []
        for d in range(W):
            o, offs = 0, []
            for f in range(F):
                offs.append(o)
                o += self.cap[d][f]
            self.seg_off.append(offs)
        # exchange A (fp32), destination block d: [gradient rows S_d x D | counts F, keys S_d (int64) | pad]
        self.Asz = [self.S[d] * D + rup(2 * (F + self.S[d]), D) for d in range(W)]
        self.A_off = [sum(self.Asz[:d]) for d in range(W)]
        self.A_total = sum(self.Asz)
        # exchange B (bf16 rows), one stride RSTR per block: [rows S | pad to Smax | tower gradient as
        # fp32 bits (2 Ppad bf16 slots)] — equal splits, and the W tower gradients at a fixed stride
        self.Smax = max(self.S)
        self.RSTR = self.Smax + 2 * self.Ppad // D
        self.RB_off = [d * self.RSTR for d in range(W)]
        if W * max(self.S) >= (1 << 18) or self.A_total // D >= 2 ** 31:
            raise _lib.TTError("sharded step: exchange too large for one step (lookups per owner < 2^18)")

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

    def grad_rows(self, parity: int) -> torch.Tensor:
        """[F * B, D] view of the gradient rows T1 wrote for the batch of this parity, in lookup
        (feature, bag) order (-1 positions: zeros) — tests."""
        pos = self.pos_out[parity].long()
        rows = self.sendA.view(-1, self.D)
        out = rows[pos.clamp(min=0)].clone()
        out[pos < 0] = 0
        return out

    def tower_grad_sent(self) -> torch.Tensor:
        """This rank's tower gradient x 1/W as sent in exchange B (tests)."""
        f = self.rows_out.view(-1).view(torch.float32)
        return f[self._tw_off[0]:self._tw_off[0] + self.towers.num_params].clone()

    def rows_for(self, parity: int) -> torch.Tensor:
        """[F * B, D] bf16 rows T1 reads for the batch of this parity (tests)."""
        pos = self.pos_in[parity].long()
        out = self.rows_in[pos.clamp(min=0)].clone()
        out[pos < 0] = 0
        return out

    def load_batch(self, cols: Sequence[torch.Tensor], labels: torch.Tensor) -> None:
        for dst, src in zip(self.cols, cols):
            dst.copy_(src, non_blocking=True)
        self.labels.copy_(labels, non_blocking=True)

    # ---- the step's pieces ----------------------------------------------------------------------
    def _route(self, cols: Sequence[torch.Tensor], parity: int) -> None:
        lib = _lib.load()
        check(lib.tt_shard_route_segs(self.F, self.B, ptr_array(list(cols)), id_dtype_code(cols[0].dtype), self._ne,
                                      self._bs, self._ow, self.W, ptr(self.segs), ptr(self.sendA),
                                      ptr(self.pos_in[parity]), ptr(self.pos_out[parity]), ptr(self.flags),
                                      ptr(self.route_ws), self.route_ws.numel(), stream_handle(self.device)),
              "shard_route_segs")

    def _exchange_a(self, stored: bool = False) -> None:
        r = self.rank
        kw = {"stored": True} if stored else {}
        self.comm.all_to_all(self.recvA, self.sendA, out_splits=[self.Asz[r]] * self.W, in_splits=list(self.Asz), **kw)

    def _gather(self, parity: int) -> None:
        check(_lib.load().tt_shard_gather_segs_bf16(*self._gather_args(parity)), "shard_gather_segs")

    def _gather_args(self, parity: int):
        r, ts = self.rank, self.tables
        ws = self.dd_ws[parity]
        return (ptr(ts.weights), ts._tm, ts.T, self.F, self.W, ptr(self.recvA), self.Asz[r] // 2,
                self.S[r] * self.D // 2, self._segoff_me, self.S[r], ptr(self.rows_out), self.RSTR,
                ptr(self.flags[1:]), ptr(ws), ws.numel(), self.max_lookups, stream_handle(self.device))

    def _exchange_b(self, stored: bool = False) -> None:
        kw = {"stored": True} if stored else {}
        self.comm.all_to_all(self.rows_in, self.rows_out, out_splits=[self.RSTR] * self.W,
                             in_splits=[self.RSTR] * self.W, **kw)

    def _t1(self, parity: int, labels: torch.Tensor, direct: bool = False) -> None:
        lib, tw, B = _lib.load(), self.towers, self.B
        pin, pout = self.pos_in[parity], self.pos_out[parity]
        if self.multi:
            check(lib.tt_tower_fwd_bwd_indexed_multi_bf16(
                C.byref(tw.shape), B, self.D, ptr(pin), ptr(pout), ptr(self.rows_in), ptr(self.sendA),
                ptr(self.params), ptr(labels), _lib.TT_I32, 1.0, ptr(self.logits), ptr(tw.ws), tw.nbytes,
                stream_handle(self.device)), "tower_fwd_bwd_indexed_multi")
            return
        check(lib.tt_tower_fwd_bwd_indexed2_bf16(
            C.byref(tw.shape), B, ptr_array([pin[:B], pin[B:]]), ptr_array([pout[:B], pout[B:]]),
            ptr_array([self.rows_in, self.rows_in]), ptr_array([self.sendA, self.sendA]), ptr(self.params),
            ptr(labels), _lib.TT_I32, 1.0, ptr(self.logits), ptr(tw.ws), tw.nbytes,
            C.byref(self._dA) if direct else None, stream_handle(self.device)),
            "tower_fwd_bwd_indexed2")

    def _rows_update(self, parity: int) -> None:
        """The owner's fused row-wise Adagrad over the received gradient rows (one pseudo-feature
        per source rank, lookups summed in ascending (source, slot) order)."""
        ts, r = self.tables, self.rank
        ws = self.dd_ws[parity]
        check(_lib.load().tt_dedup_rowwise_adagrad(ts._tm, ts.T, self._fm_src, self.W, self.S[r], ptr(self.recvA),
                                                  self.D, ptr(ts.weights), ptr(ts.state), self.lr_emb, self.eps,
                                                  ptr(ws), ws.numel(), self.max_lookups, stream_handle(self.device)),
              "dedup_rowwise_adagrad")

    def _adam(self, wait=None) -> None:
        """Adam on the fixed-order sum of the W tower gradients received in exchange B, with the
        step scalars T2 wrote (launch U / tt_tower_wgrad_pre advanced the step). ``wait``: exchange
        B's in-launch signal / wait (tt_peer_wait_t)."""
        tw = self.towers
        grads = self.rows_in.data_ptr() + 4 * self._tw_in
        check(_lib.load().tt_tower_adam_pre_grads_sum(
            C.byref(tw.shape), self.B, ptr(self.params), grads, self.W, self._tw_stride, ptr(self.exp_avg),
            ptr(self.exp_avg_sq), 1e-8, 0.9, 0.999, 0.0, ptr(tw.ws), tw.nbytes,
            C.byref(wait) if wait is not None else None, stream_handle(self.device)), "tower_adam_pre_grads_sum")

    def _plan(self, roles: int, route, ws: torch.Tensor, wait: bool = False) -> "_lib.LaunchPlan":
        """A tt_launch plan for the pipelined step's launches U / G: the towers, the WGRAD role, the
        route of a later batch (``route`` = _route_args) and the owner's ADAGRAD role over the received
        gradient rows (one pseudo-feature per source rank) in dedup workspace ``ws``; ``wait``:
        launch U signals / waits exchange A in-launch."""
        tw, ts, r = self.towers, self.tables, self.rank
        return _lib.LaunchPlan(
            wait=C.pointer(self._wA) if wait else None,
            roles=roles, shape=C.pointer(tw.shape), B=self.B, workspace=ptr(tw.ws), ws_bytes=tw.nbytes,
            wgrad=_lib.WgradRole(loss=ptr(self.loss), adam_step_state=ptr(self.adam_state), adam_lr=self.lr_dense,
                                 adam_beta1=0.9, adam_beta2=0.999),
            route=_lib.RouteRole(F=route[0], cols=route[1], id_dtype=route[2], num_embeddings=route[3],
                                 block_sizes=route[4], owners=route[5], W=route[6], segs=route[7], send=route[8],
                                 pos_in=route[9], pos_out=route[10], overflow=route[11], route_ws=route[12],
                                 route_ws_bytes=route[13]),
            adagrad=_lib.AdagradRole(tables=ts._tm, T=ts.T, F=self.W, features=self._fm_src, B=self.S[r],
                                     grad=ptr(self.recvA), ldg=self.D, weights=ptr(ts.weights), state=ptr(ts.state),
                                     lr=self.lr_emb, eps=self.eps, dedup_ws=ptr(ws), dedup_ws_bytes=ws.numel(),
                                     dedup_max_lookups=self.max_lookups, multi_only=0))

    def _route_args(self, cols: Sequence[torch.Tensor], parity: int):
        return (self.F, ptr_array(list(cols)), id_dtype_code(cols[0].dtype), self._ne, self._bs, self._ow, self.W,
                ptr(self.segs), ptr(self.sendA), ptr(self.pos_in[parity]), ptr(self.pos_out[parity]),
                ptr(self.flags), ptr(self.route_ws), self.route_ws.numel())

    # ---- public steps ---------------------------------------------------------------------------
    def step(self) -> None:
        """One synchronous step on the batch in ``cols`` / ``labels`` (no later batch known: ids,
        rows, gradient rows and tower gradients each take an exchange)."""
        lib, tw = _lib.load(), self.towers
        if self.cursor is not None:  # a pipelined run left batches staged in the dedup tables
            self.reset_pipeline()
        self._route(self.cols, 0)
        self._exchange_a()
        self._gather(0)
        self._exchange_b()
        self._t1(0, self.labels)
        check(lib.tt_tower_wgrad_pre(C.byref(tw.shape), self.B, ptr(self.loss), ptr(tw.ws), tw.nbytes,
                                     ptr(self.adam_state), self.lr_dense, 0.9, 0.999, None, 0, 0,
                                     stream_handle(self.device)), "tower_wgrad_pre")
        check(lib.tt_tower_grads_replicated(C.byref(tw.shape), self.B, ptr(self.params),
                                            self.rows_out.data_ptr(), self.W, self._tw_off, 1.0 / self.W, ptr(tw.ws),
                                            tw.nbytes, stream_handle(self.device)), "tower_grads_replicated")
        self._exchange_a()
        self._rows_update(0)
        self._exchange_b()
        self._adam()

    def prime(self, cols: Sequence[torch.Tensor], parity: int, next_cols: Optional[Sequence[torch.Tensor]] = None) -> None:
        """Stage the rows of a batch (the pipelined loop's first step) and, with ``next_cols``, place
        the following batch's keys (its route, parity ^ 1). Starts from empty dedup tables (a
        second prime over staged state would file the same keys twice)."""
        self.reset_pipeline()
        self._route(cols, parity)
        self._exchange_a()
        self._gather(parity)
        self._exchange_b()
        if next_cols is not None:
            self._route(next_cols, parity ^ 1)

    def step_pipelined(self, labels: torch.Tensor, parity: int, next2_cols: Sequence[torch.Tensor]) -> None:
        """Step on the staged batch i (rows in place, parity ``parity``; batch i+1's keys placed),
        staging batch i+1's rows and routing ``next2_cols`` (batch i+2, same parity)."""
        lib, tw, ts, r, B, dev = _lib.load(), self.towers, self.tables, self.rank, self.B, self.device
        direct, merged = self.direct, self.merged
        self._t1(parity, labels, direct=direct)
        route = self._route_args(next2_cols, parity)
        ws = self.dd_ws[parity]
        main = torch.cuda.current_stream(dev)
        if self.overlap:
            # T2 (weight gradients + Adam's step scalars) on a parallel branch: it reads only T1's
            # operand strips, so it overlaps exchange A and the owner's update; launch G (which
            # reduces T2's slabs into exchange B) joins it
            self.side.wait_stream(main)
            with torch.cuda.stream(self.side):
                check(lib.tt_tower_wgrad_pre(C.byref(tw.shape), B, ptr(self.loss), ptr(tw.ws), tw.nbytes,
                                             ptr(self.adam_state), self.lr_dense, 0.9, 0.999, None, 0, 0,
                                             stream_handle(dev)), "tower_wgrad_pre")
            if not merged:
                self._exchange_a(stored=direct)
            # launch U without T2: the owner's row-wise Adagrad + the count pass of batch i+2's route
            _lib.launch(self._plan(_lib.ROLE_ROUTE_COUNT | _lib.ROLE_ADAGRAD, route, ws, merged), stream_handle(dev),
                        "shard_route_count_rowwise_adagrad")
            main.wait_stream(self.side)
        else:
            if not merged:
                self._exchange_a(stored=direct)
            # launch U: T2 + the count pass of batch i+2's route + the owner's row-wise Adagrad
            _lib.launch(self._plan(_lib.ROLE_WGRAD | _lib.ROLE_ROUTE_COUNT | _lib.ROLE_ADAGRAD, route, ws, merged),
                        stream_handle(dev), "tower_wgrad_route_count_rowwise_adagrad")
        # launch G: the tower gradient x 1/W into every destination block + the route's place pass +
        # the owner's gather of batch i+1's rows
        plan = self._plan(_lib.ROLE_UPDATE | _lib.ROLE_ROUTE_PLACE | _lib.ROLE_GATHER, route, ws)
        plan.update = _lib.UpdateRole(params=ptr(self.params), replicated=1, copies=self.W,
                                      base=self.rows_out.data_ptr(),
                                      offsets=self._tw_off_direct if direct else self._tw_off, scale=1.0 / self.W)
        g = self._gather_args(parity ^ 1)
        plan.gather = _lib.GatherRole(weights=g[0], tables=g[1], T=g[2], recv=g[5], block_i64=g[6], counts_i64=g[7],
                                      seg_off=g[8], slots=g[9], rows_out=g[10], out_stride=g[11], bad=g[12],
                                      dedup_ws=g[13], dedup_ws_bytes=g[14], dedup_max_lookups=g[15],
                                      direct=C.pointer(self._dB) if direct else None)
        _lib.launch(plan, stream_handle(dev), "tower_grads_replicated_route_place_gather")
        if merged:
            self._adam(self._wB)
        else:
            self._exchange_b(stored=direct)
            self._adam()

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

    def _names(self, feature_names):
        names = list(feature_names) if feature_names is not None else (
            ["user_id", "product_id"] if self.F == 2 else [f"f{i}" for i in range(self.F)])
        if len(names) != self.F:
            raise _lib.TTError("one feature name per feature")
        return names

    def gathered_state_dict(self, feature_names: Optional[Sequence[str]] = None,
                            prefix: str = "two_tower.", optimizer: bool = False) -> Dict[str, torch.Tensor]:
        """Collective: rank 0 returns the full state dict the reference's gather_and_get_state_dict
        writes (full tables + towers), other ranks {}. ``optimizer``: also the row-wise Adagrad state
        of every table (gathered like the tables) and the towers' Adam moments and step under
        ``optim.*`` keys (the reference saves no optimizer state; this makes resume exact)."""
        from .lifecycle import _dense_items, _tower_views

        sd = {}
        for f, name in enumerate(self._names(feature_names)):
            full = self.comm.gather_rows(self.tables.table_view(f), self.spans(f), self.N[f])
            if self.rank == 0:
                sd[f"{prefix}ebc.embedding_bags.t_{name}.weight"] = full
            if optimizer:
                st = self.comm.gather_rows(self.tables.state_view(f).unsqueeze(1), self.spans(f), self.N[f])
                if self.rank == 0:
                    sd[f"optim.ebc.t_{name}.rowwise_adagrad_state"] = st[:, 0].clone()
        if self.rank == 0:
            towers = _tower_views(self.params, self.in_dims, self.layer_sizes)
            sd.update({k: v.clone() for k, v in _dense_items(towers, prefix).items()})
            if optimizer:
                sd["optim.towers.exp_avg"] = self.exp_avg.clone()
                sd["optim.towers.exp_avg_sq"] = self.exp_avg_sq.clone()
                sd["optim.towers.step"] = self.adam_state[:1].clone()
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor], feature_names: Optional[Sequence[str]] = None,
                        prefix: str = "two_tower.") -> None:
        """Every rank takes its blocks of the full tables and the towers from a gathered dict (and
        the optimizer state when the dict holds ``optim.*`` keys; otherwise it is reset)."""
        from .lifecycle import _dense_items, _tower_views

        with torch.no_grad():
            for f, name in enumerate(self._names(feature_names)):
                lo, n = self.spans(f)[self.rank]
                if n:
                    self.tables.table_view(f)[:n].copy_(sd[f"{prefix}ebc.embedding_bags.t_{name}.weight"][lo:lo + n])
                    key = f"optim.ebc.t_{name}.rowwise_adagrad_state"
                    if key in sd:
                        self.tables.state_view(f)[:n].copy_(sd[key][lo:lo + n])
                    else:
                        self.tables.state_view(f).zero_()
            towers = _tower_views(self.params, self.in_dims, self.layer_sizes)
            for k, v in _dense_items(towers, prefix).items():
                v.copy_(sd[k])
            if "optim.towers.exp_avg" in sd:
                self.exp_avg.copy_(sd["optim.towers.exp_avg"])
                self.exp_avg_sq.copy_(sd["optim.towers.exp_avg_sq"])
                self.adam_state.zero_()
                self.adam_state[:1].copy_(sd["optim.towers.step"])
            else:
                self.exp_avg.zero_()
                self.exp_avg_sq.zero_()
                self.adam_state.zero_()
        self.towers.update(self.params, do_adam=False)
        # rows staged before the load are stale, and the dedup tables were filed for them: the next
        # pipelined run (graph replay or eager) primes again from the loaded weights
        self.reset_pipeline()

    def check(self, collective: bool = True) -> None:
        """Raise if any step so far overflowed a segment or received a key outside its shard. With
        ``collective`` (default) the flags are first max-reduced over the ranks, so every rank
        raises together (call it on every rank, outside any graph capture)."""
        f = self.flags.clone()
        perr = getattr(self.comm, "err", None)  # PeerComm: a wait that timed out
        if perr is not None:
            f = torch.cat([f, perr])
        if collective:
            self.comm.all_reduce_max_(f)
        f = f.cpu().tolist()
        if len(f) > 2 and f[2]:
            raise _lib.TTError("sharded step: a device-initiated exchange timed out waiting for a peer: results are "
                               "invalid")
        if f[0]:
            raise _lib.TTError(f"sharded step: a segment exceeded its capacity {self.caps_f} (skewed ids): "
                               "results are invalid; raise `capacity`")
        if f[1]:
            raise _lib.TTError("sharded step: an owner received a key outside its shard")

    def release_graphs(self) -> None:
        """Drop the captured graphs (before tearing down the process group: a live graph holds
        references to the RCCL communicator's work)."""
        torch.cuda.synchronize(self.device)
        self.pool_graphs = []
        self.small_graphs = []
        self._pool_inputs = []
        import gc

        gc.collect()
        torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------------------------------
    def _staged(self, batches: Sequence) -> list:
        staged = []
        for cols, labels in batches:
            cols = list(cols)
            if len(cols) != self.F:
                raise _lib.TTError("capture_pool: one id column per feature expected")
            for c in cols:
                if c.dtype != self.id_dtype or not c.is_contiguous() or c.numel() != self.B or c.device != self.device:
                    raise _lib.TTError("capture_pool: batch columns must be contiguous [B] device tensors of the "
                                       "step's id dtype")
            lab = labels.to(torch.int32).contiguous()
            if lab.numel() != self.B:
                raise _lib.TTError("capture_pool: labels must be [B]")
            staged.append((cols, lab))
        return staged

    def capture_pool(self, batches: Sequence, steps_per_graph: int = 1) -> None:
        """Pipelined HIP graphs over a cyclic pool of resident (cols, labels) batches (len even, a
        multiple of k = ``steps_per_graph``): graph j runs the steps of batches j*k .. j*k+k-1, each
        staging the next batch of the pool; ``small_graphs[i]`` runs batch i alone. Replay them in
        pool order with ``run(n)`` (the step keeps the cursor). Needs a capturable comm."""
        if not self.comm.capturable:
            raise _lib.TTError("capture_pool: the comm is not graph-capturable")
        k = int(steps_per_graph)
        n = len(batches)
        if k < 1 or n % k or n % 2:
            raise _lib.TTError("capture_pool: the batch count must be even and a multiple of steps_per_graph")
        staged = self._staged(batches)
        self._pool_inputs = [staged]
        self.pool_k = k
        self._prefault_due = True  # the next replay walks the tables' pages first (TableSet.prefault)
        # stage batch 0 (and place batch 1's keys) eagerly, then retire every eager collective
        self.prime(staged[0][0], 0, staged[1][0])
        self.cursor = 0
        self.comm.retire()

        def cap(idx):
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    for i in idx:
                        self.step_pipelined(staged[i][1], i % 2, staged[(i + 2) % n][0])
            torch.cuda.current_stream(self.device).wait_stream(s)
            _lib.graph_upload(g, self.device)  # no upload inside the first (timed) launch
            return g

        torch.cuda.synchronize(self.device)
        self.pool_graphs = [cap(range(j, j + k)) for j in range(0, n, k)]
        self.small_graphs = [cap([i]) for i in range(n)] if k > 1 else list(self.pool_graphs)
        torch.cuda.synchronize(self.device)

    def run(self, n: int) -> None:
        """Replay n pipelined steps from the pool, continuing at the cursor (re-primed at the pool's
        first batch after ``reset_pipeline`` / ``load_state_dict``)."""
        if getattr(self, "_prefault_due", False):  # first replay after a capture: the tables' pages
            self._prefault_due = False  # walked right before it (TableSet.prefault; r06pf_* profiles)
            self.tables.prefault()
        if not self.small_graphs:
            raise _lib.TTError("run: no captured pool (capture_pool first)")
        if self.cursor is None:
            staged = self._pool_inputs[0]
            self.prime(staged[0][0], 0, staged[1][0])
            self.cursor = 0
        i, nb, k = self.cursor, len(self.small_graphs), self.pool_k
        while n > 0:
            if i % k == 0 and n >= k:
                self.pool_graphs[i // k].replay()
                i, n = i + k, n - k
            else:
                self.small_graphs[i].replay()
                i, n = i + 1, n - 1
            i %= nb
        self.cursor = i

    def run_eager(self, batches: Sequence, n: int) -> None:
        """n pipelined steps over a cyclic pool without graphs (continuing at the cursor)."""
        nb = len(batches)
        if nb % 2:
            raise _lib.TTError("run_eager: the pool needs an even number of batches")
        if self.cursor is None:
            self.prime(list(batches[0][0]), 0, list(batches[1][0]))
            self.cursor = 0
        for _ in range(n):
            i = self.cursor
            self.step_pipelined(batches[i][1].to(torch.int32), i % 2, list(batches[(i + 2) % nb][0]))
            self.cursor = (i + 1) % nb


def capture_pool_or_eager(step: FusedShardedTwoTowerStep, batches: Sequence, steps_per_graph: int,
                          allow_capture: bool = True) -> str:
    """Collective (every rank): capture the pipelined pool into HIP graphs, or fall back to eager
    steps on EVERY rank when any rank's capture is refused (or ``allow_capture`` is off, e.g. gloo
    collectives). The fallback drops the graphs and the staged state the capture primed, so the
    eager run starts from clean dedup tables. Returns "hipgraph" or "eager"."""
    ok = torch.ones(1, device=step.device)
    if allow_capture:
        try:
            step.capture_pool(batches, steps_per_graph=steps_per_graph)
        except Exception as e:  # noqa: BLE001 - the same work per step runs eagerly
            import sys

            print(f"rank {step.rank}: graph capture with collectives refused ({e}); eager steps", file=sys.stderr)
            ok.zero_()
    else:
        ok.zero_()
    torch.cuda.synchronize(step.device)
    if dist.is_initialized():
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)  # every rank takes the same mode
    if float(ok) >= 1:
        return "hipgraph"
    step.release_graphs()
    step.reset_pipeline()
    if dist.is_initialized():
        dist.barrier()
    return "eager"
