"""Host logic of the device-initiated exchange (sharded.PeerComm.all_to_all, no GPU): where each block of
the send buffer goes — peer d's receive buffer at this rank's slot, its flag word for this source — and
the argument checks, with the library's exchange call replaced by a recorder."""
import ctypes as C
import types

import pytest
import torch

from two_tower_recommender_model_amd import _lib, sharded


class _Rec:
    def __init__(self):
        self.puts, self.waits = [], []

    def tt_peer_exchange(self, p, flags, err, timeout, stream):
        self.puts.append(C.cast(p, C.POINTER(_lib.PeerPut)).contents)
        self.waits.append((flags, err, timeout))
        return 0


def _comm(monkeypatch, W, rank, peers, out):
    rec = _Rec()
    monkeypatch.setattr(_lib, "load", lambda path=None: rec)
    monkeypatch.setattr(sharded, "stream_handle", lambda device=None: 0)
    pc = object.__new__(sharded.PeerComm)
    pc.world, pc.rank, pc.timeout_s, pc.same_device, pc.shared_gpu = W, rank, 5.0, False, False
    pc.err = torch.zeros(1, dtype=torch.int32)
    pc._puts = {}
    pc._bufs = {out.data_ptr(): {"peers": peers, "flags": torch.zeros(W, dtype=torch.int32),
                                 "state": torch.zeros(1, dtype=torch.int32)}}
    return pc, rec


def test_blocks_land_at_this_ranks_slot_of_every_peer(monkeypatch):
    W, r = 3, 1
    sizes = [8, 4, 12]  # rows sent to each destination (1-D fp32: a row is 4 B)
    inp = torch.zeros(sum(sizes) + 4)
    out = torch.zeros(W * sizes[r])
    peers = [(1 << 20, 4096), (2 << 20, 8192), (3 << 20, 1024)]
    pc, rec = _comm(monkeypatch, W, r, peers, out)
    pc.all_to_all(out, inp, out_splits=[sizes[r]] * W, in_splits=sizes)
    (p,) = rec.puts
    assert (p.W, p.rank, p.src) == (W, r, inp.data_ptr())
    off = 0
    for d in range(W):
        assert p.src_off[d] == off * 4 and p.len[d] == sizes[d] * 4
        assert p.dst[d] == peers[d][0] + r * sizes[d] * 4  # peer d receives equal blocks of sizes[d] rows
        assert p.flag[d] == peers[d][0] + peers[d][1] + 4 * r
        off += sizes[d]
    assert rec.waits[0][2] == 5.0 and p.same_device == 0
    pc.all_to_all(out, inp, out_splits=[sizes[r]] * W, in_splits=sizes)
    assert len(pc._puts) == 1 and len(rec.puts) == 2  # the put arguments are built once per exchange


def test_equal_blocks_of_rows(monkeypatch):
    W, r, rows, D = 2, 0, 6, 8
    inp = torch.zeros(W * rows, D, dtype=torch.bfloat16)
    out = torch.zeros(W * rows, D, dtype=torch.bfloat16)
    peers = [(1 << 20, 256), (5 << 20, 512)]
    pc, rec = _comm(monkeypatch, W, r, peers, out)
    pc.all_to_all(out, inp)
    (p,) = rec.puts
    rowb = D * 2
    assert [p.src_off[d] for d in range(W)] == [0, rows * rowb]
    assert [p.len[d] for d in range(W)] == [rows * rowb] * W
    assert [p.dst[d] for d in range(W)] == [peers[d][0] for d in range(W)]  # rank 0's slot is block 0


def test_rejects_foreign_and_mismatched_buffers(monkeypatch):
    W, r = 2, 0
    out = torch.zeros(8)
    pc, _ = _comm(monkeypatch, W, r, [(1 << 20, 64), (2 << 20, 64)], out)
    with pytest.raises(_lib.TTError, match="recv_buffer"):
        pc.all_to_all(torch.zeros(8), torch.zeros(8))
    with pytest.raises(_lib.TTError, match="do not match"):
        pc.all_to_all(out, torch.zeros(16), out_splits=[4, 4], in_splits=[6, 2])  # 6 sent to self, 4 expected
    with pytest.raises(_lib.TTError, match="equal receive blocks"):
        pc.all_to_all(out, torch.zeros(8), out_splits=[3, 5], in_splits=[4, 4])


def test_torch_and_thread_comms_give_plain_receive_buffers():
    t = types.SimpleNamespace()
    b = sharded.TorchComm.recv_buffer(t, (4, 2), torch.float32, "cpu")
    assert b.shape == (4, 2) and not b.any()
    th = sharded.ThreadComm.group(1)[0]
    assert th.recv_buffer((3,), torch.bfloat16, "cpu").dtype == torch.bfloat16


def test_stored_exchange_signals_only(monkeypatch):
    """stored=True (the producers wrote the blocks themselves): a descriptor of the same flags and
    destinations with every length 0 — tt_peer_exchange then runs only its signal / wait kernel."""
    W, r = 2, 1
    sizes = [8, 4]
    inp = torch.zeros(sum(sizes))
    out = torch.zeros(W * sizes[r])
    peers = [(1 << 20, 4096), (2 << 20, 8192)]
    pc, rec = _comm(monkeypatch, W, r, peers, out)
    pc.all_to_all(out, inp, out_splits=[sizes[r]] * W, in_splits=sizes, stored=True)
    (p,) = rec.puts
    assert [p.len[d] for d in range(W)] == [0, 0]
    assert [p.flag[d] for d in range(W)] == [peers[d][0] + peers[d][1] + 4 * r for d in range(W)]
    pc.all_to_all(out, inp, out_splits=[sizes[r]] * W, in_splits=sizes)
    assert rec.puts[1].len[0] == sizes[0] * 4 and len(pc._puts) == 2  # put and signal-only cached apart


def test_direct_descriptor_addresses_rows_and_copies(monkeypatch):
    """PeerComm.direct: block d of the send buffer starts at unit first_row[d] and lands at peer d's
    buffer at this rank's slot (row0[d]); the copy range of block d goes to the same place + lo."""
    W, r, D = 3, 2, 4
    rows = [16, 8, 24]  # units (rows of D floats) per destination block
    inp = torch.zeros(sum(rows), D)
    out = torch.zeros(W * rows[r], D)
    peers = [(1 << 24, 65536), (2 << 24, 65536), (3 << 24, 65536)]
    pc, _ = _comm(monkeypatch, W, r, peers, out)
    rowb = 4 * D
    x = pc.direct(out, inp, rowb, out_splits=[rows[r]] * W, in_splits=rows,
                  copy=[(rowb * (n - 2), rowb * n) for n in rows])  # the last two rows of each block
    assert x.W == W
    o = 0
    for d in range(W):
        assert x.first_row[d] == o
        assert x.row0[d] == peers[d][0] + r * rows[d] * rowb
        assert x.copy_src[d] == inp.data_ptr() + (o + rows[d] - 2) * rowb
        assert x.copy_dst[d] == x.row0[d] + (rows[d] - 2) * rowb and x.copy_len[d] == 2 * rowb
        o += rows[d]
    with pytest.raises(_lib.TTError, match="16-B aligned"):
        pc.direct(out, inp, rowb, out_splits=[rows[r]] * W, in_splits=rows, copy=[(4, 16)] * W)
    with pytest.raises(_lib.TTError, match="do not match"):
        pc.block_dst(out, inp, out_splits=[rows[r] + 1] * W, in_splits=rows)


def test_in_launch_wait_descriptor(monkeypatch):
    """PeerComm.wait_desc (tt_peer_wait_t): the consumer signals peer d's flag word for this source and
    polls this rank's W flag words against the exchange's epoch word — the one the producer's
    descriptor (direct(..., epoch=True)) advances; refused when the ranks share a GPU."""
    W, r, D = 3, 1, 4
    rows = [8, 8, 8]
    inp = torch.zeros(sum(rows), D)
    out = torch.zeros(W * rows[r], D)
    peers = [(1 << 24, 4096), (2 << 24, 8192), (3 << 24, 1024)]
    pc, _ = _comm(monkeypatch, W, r, peers, out)
    e = pc._bufs[out.data_ptr()]
    x = pc.direct(out, inp, 4 * D, epoch=True)
    assert x.epoch == e["state"].data_ptr() and not pc.direct(out, inp, 4 * D).epoch
    assert pc.in_launch_wait
    w = pc.wait_desc(out)
    assert (w.W, w.sys) == (W, 1)
    assert [w.flag[d] for d in range(W)] == [peers[d][0] + peers[d][1] + 4 * r for d in range(W)]
    assert (w.flags, w.epoch, w.err) == (e["flags"].data_ptr(), e["state"].data_ptr(), pc.err.data_ptr())
    assert w.timeout_ticks == int(5.0 * 1e8)
    with pytest.raises(_lib.TTError, match="recv_buffer"):
        pc.wait_desc(torch.zeros(4))
    pc.shared_gpu = True  # ranks on one GPU (the scope may still be forced to system): kernels only
    assert not pc.in_launch_wait
    with pytest.raises(_lib.TTError, match="share a device"):
        pc.wait_desc(out)
    pc.world = 1
    assert pc.in_launch_wait


def test_exchange_comm_falls_back_to_rccl_when_the_self_test_fails(monkeypatch):
    """exchange_comm("auto"): a failed PeerComm self-test (on any rank: the result is agreed on)
    gives TorchComm on every rank; "peer" raises instead; "rccl" never builds a PeerComm."""
    made = []

    class FakePeer:
        def __init__(self, group=None, device=None):
            made.append(self)
            self.closed = False
            self.memory = "fine-grained"

        def self_test(self):
            return False, "rank 1: round 0: 3 of 64 received words differ"

        def close(self):
            self.closed = True

    class FakeTorch:
        def __init__(self, group=None, always_collective=False):
            self.always = always_collective

    monkeypatch.setattr(sharded, "PeerComm", FakePeer)
    monkeypatch.setattr(sharded, "TorchComm", FakeTorch)
    monkeypatch.setattr(sharded.dist, "get_rank", lambda group=None: 0)
    comm, desc = sharded.exchange_comm("auto")
    assert isinstance(comm, FakeTorch) and comm.always and made[-1].closed
    assert desc.startswith("RCCL") and "differ" in desc
    with pytest.raises(_lib.TTError, match="self-test failed"):
        sharded.exchange_comm("peer")
    n = len(made)
    comm, desc = sharded.exchange_comm("rccl")
    assert isinstance(comm, FakeTorch) and len(made) == n
    FakePeer.self_test = lambda self: (True, "")
    comm, desc = sharded.exchange_comm("auto")
    assert isinstance(comm, FakePeer) and desc.startswith("device-initiated")
    # the probe (auto, RCCL backend, block sizes given): RCCL kept when the device-initiated
    # exchange is more than 10 % slower, never probed for "peer" or without sizes
    monkeypatch.setattr(sharded.dist, "get_backend", lambda group=None: "nccl")
    times = {"t": (2.0, 1.0)}
    probed = []

    def fake_probe(pc, group, device, sizes, iters=10):
        probed.append(list(sizes))
        return times["t"]

    monkeypatch.setattr(sharded, "_probe_exchanges", fake_probe)
    comm, desc = sharded.exchange_comm("auto", probe=[1024, 512])
    assert isinstance(comm, FakeTorch) and made[-1].closed and "2000.0 us" in desc and probed == [[1024, 512]]
    times["t"] = (1.05, 1.0)
    comm, desc = sharded.exchange_comm("auto", probe=[1024])
    assert isinstance(comm, FakePeer) and "probe 1050.0 us" in desc
    n = len(probed)
    comm, _ = sharded.exchange_comm("peer", probe=[1024])
    comm2, _ = sharded.exchange_comm("auto")
    assert isinstance(comm, FakePeer) and isinstance(comm2, FakePeer) and len(probed) == n
