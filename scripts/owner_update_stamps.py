"""EXPERIMENT: per-phase wall time (s_memrealtime, 100 MHz) of the owner's row-wise Adagrad in the
pipelined sharded step's launch U (TT_DD_STAMPS): 0 start, 1 slot + meta in, 2 gradient rows
summed, 3 stores issued; slot workgroups only (the hot-row workgroups stamp 0). World 1 over an
in-process comm, north-star shape."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["TT_DD_STAMPS"] = "1"
import torch  # noqa: E402

from two_tower_recommender_model_amd.sharded import FusedShardedTwoTowerStep, ThreadComm  # noqa: E402


def dbg_offset(L):
    al = lambda x: -(-x // 256) * 256  # noqa: E731
    cap = 1024
    while cap < 16 * L:
        cap <<= 1
    off = al(128 * cap) + al(8 * L) + al(4 * (L // 31 + 1)) + al(16) + al(4 * L) + al(16 * 64 * ((L + 63) // 64))
    return off, cap


dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
N, B = [50_000_000, 100_000_000], 8192
st = FusedShardedTwoTowerStep(ThreadComm.group(1)[0], N, 128, [128, 64], B, dev)
g = torch.Generator(device=dev).manual_seed(1)
pool = [([torch.randint(0, n, (B,), generator=g, device=dev) for n in N],
         torch.randint(0, 2, (B,), generator=g, device=dev, dtype=torch.int32)) for _ in range(8)]
L = st.max_lookups
off, cap = dbg_offset(L)
hot_wgs = min(64, max(1, L // 31))
for it in range(6):
    p = (st.cursor or 0) % 2 if st.cursor is not None else 0
    st.run_eager(pool, 1)
    torch.cuda.synchronize()
    if it < 2:
        continue
    ws = st.dd_ws[p]
    n = (L // 32 + 64)
    stm = ws[off:off + 8 * 8 * n].view(torch.int64).view(n, 8)[:, :4].cpu().double()
    slot = stm[hot_wgs:]
    slot = slot[slot[:, 0] > 0]
    t0 = stm[stm[:, 0] > 0, 0].min()
    rel = (slot - t0) / 100.0
    med = lambda x: float(x.median())  # noqa: E731
    print(f"it{it} slot wgs {len(slot)}: start {med(rel[:, 0]):.2f}/{float(rel[:, 0].max()):.2f} | slot+meta "
          f"{med(rel[:, 1]):.2f} | grads {med(rel[:, 2]):.2f} | stores {med(rel[:, 3]):.2f}/{float(rel[:, 3].max()):.2f}")
