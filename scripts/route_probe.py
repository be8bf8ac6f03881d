"""Probe: device time of the sharded route kernels (two-kernel uniform form vs the single-launch
segment form) at B = 8192, F = 2, for W in {1, 8}; run under rocprofv3 --kernel-trace --stats."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from two_tower_recommender_model_amd import _lib  # noqa: E402
from two_tower_recommender_model_amd._lib import ShardSeg, ptr, ptr_array, stream_handle  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
B, F = 8192, 2
N = [50_000_000, 100_000_000]
for W in (1, 8):
    cols = [torch.randint(0, n, (B,), device=dev) for n in N]
    bs = [-(-n // W) for n in N]
    C_ = B if W == 1 else 1344
    send = torch.zeros(W * (F + F * C_) * 2, dtype=torch.int64, device=dev)
    pos = torch.zeros(F * B, dtype=torch.int32, device=dev)
    pos2 = torch.zeros(F * B, dtype=torch.int32, device=dev)
    flags = torch.zeros(2, dtype=torch.int32, device=dev)
    ws = torch.empty(lib.tt_shard_route_workspace_bytes(F, B), dtype=torch.uint8, device=dev)
    segs = (ShardSeg * (W * F))()
    for d in range(W):
        for f in range(F):
            e = segs[d * F + f]
            e.cap, e.key_index, e.cnt_index = C_, (d * F + f) * C_ + W * F, d * F + f
            e.pos_in, e.pos_out = (d * F + f) * C_, (d * F + f) * C_
    segs_d = torch.frombuffer(bytearray(bytes(segs)), dtype=torch.uint8).to(dev)
    ne, bsz, ow = (C.c_int64 * F)(*N), (C.c_int64 * F)(*bs), (C.c_int32 * F)(0, 0)
    st = stream_handle(dev)
    for _ in range(20):
        _lib.check(lib.tt_shard_route_cols(F, B, ptr_array(cols), 1, ne, bsz, ow, W, C_, ptr(send), ptr(pos), ptr(flags),
                                           ptr(ws), ws.numel(), st))
        _lib.check(lib.tt_shard_route_segs(F, B, ptr_array(cols), 1, ne, bsz, ow, W, ptr(segs_d), ptr(send), ptr(pos),
                                           ptr(pos2), ptr(flags), ptr(ws), ws.numel(), st))
    torch.cuda.synchronize()
    print("W", W, "flags", flags.tolist())
