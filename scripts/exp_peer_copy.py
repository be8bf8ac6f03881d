"""EXPERIMENT: the device-initiated exchange (sharded.PeerComm) in isolation at world 1 — an
all-to-all of the sharded step's exchange-A size (8.5 MB) and exchange-B size (4.2 MB), timed with
HIP events over back-to-back calls, against torch's copy_ of the same bytes and RCCL's
all_to_all_single. Memory modes: fine-grained (default) and the torch allocator (TT_PEER_MEMORY)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from two_tower_recommender_model_amd.sharded import PeerComm  # noqa: E402


def timed(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(), device_id=dev)
    for mem in ("fine-grained", "device"):
        pc = PeerComm(device=dev, memory=mem)
        for name, nbytes in (("A", 8_520_192), ("B", 4_194_304)):
            n = nbytes // 4
            inp = torch.randn(n, device=dev)
            out = pc.recv_buffer((n,), torch.float32, dev)
            plain = torch.empty(n, device=dev)
            t_peer = timed(lambda: pc.all_to_all(out, inp))
            assert torch.equal(out, inp)
            t_copy = timed(lambda: plain.copy_(inp))
            t_copy_to = timed(lambda: out.copy_(inp))
            t_rccl = timed(lambda: dist.all_to_all_single(plain, inp))
            print(f"{mem:13s} {name} {nbytes / 1e6:.1f} MB: peer {t_peer:6.2f} us | torch copy_ {t_copy:6.2f} us "
                  f"(into the peer buffer {t_copy_to:6.2f}) | RCCL all_to_all_single {t_rccl:6.2f} us", flush=True)
        pc.close()
    dist.destroy_process_group()
    time.sleep(0.1)


if __name__ == "__main__":
    main()
