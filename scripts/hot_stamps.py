"""EXPERIMENT: phases of the hot-row role (dd_hot_role) and, with LIST=1, of the list role (dd_multi_block:
0 start, 2 rows summed, 3 stores issued, per update workgroup 64..191) inside the ring's tail launch at Zipf ids
(TT_DD_STAMPS; experiment library: `TT_EXTRA_CFLAGS=-DDD_HOT_STAMPS=1 python -m
two_tower_recommender_model_amd.build --experiments`, run with TT_EXPERIMENT_LIB=1): per hot
workgroup, s_memrealtime (100 MHz) at 4 first pass scanned, 5 passes summed,
6 partial published + counter added, 7 row update issued; us from the workgroup's start."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["TT_DD_STAMPS"] = "1"
os.environ.setdefault("TT_EXPERIMENT_LIB", "1")
import torch  # noqa: E402

from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402

dev = torch.device("cuda:0")
N = [50_000_000, 100_000_000]
B = 8192
st = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, dev)
g = torch.Generator(device=dev).manual_seed(1)


def ids(n):
    u01 = torch.rand(B, generator=g, device=dev, dtype=torch.float64)
    r = torch.floor(torch.exp(u01 * torch.log(torch.tensor(float(n), device=dev, dtype=torch.float64))))
    return (r.to(torch.int64) * 2654435761) % n


batches = [([ids(n) for n in N], torch.randint(0, 2, (B,), generator=g, device=dev, dtype=torch.int32))
           for _ in range(64)]
st.capture_ring(batches, steps_per_graph=8)


def a256(x):
    return (x + 255) // 256 * 256


L = st.tables._dd_cap
cap = 1024
while cap < 16 * L:
    cap <<= 1
off = a256(cap * 128) + a256(8 * L) + a256(4 * (L // 31 + 1)) + a256(16) + a256(4 * L) + a256(16 * 64 * ((L + 63) // 64))
NW = 192 if os.environ.get("LIST") else 64
for it in range(4):
    for w in st._ring:
        w[off:off + 8 * 8 * NW].zero_()
    st.run_eager(1)
    torch.cuda.synchronize()
    if it < 2:
        continue
    for w in st._ring:
        if NW > 64:
            sl = w[off + 8 * 8 * 64:off + 8 * 8 * NW].view(torch.int64).view(NW - 64, 8).cpu().double()
            sl = sl[sl[:, 3] != 0]
            if len(sl):
                t0 = float(sl[:, 0].min())
                rel = (sl - sl[:, :1]) / 100.0
                print(f"list wgs {len(sl)}: start p50/max {float(((sl[:, 0] - t0) / 100).median()):.2f}/"
                      f"{float(((sl[:, 0] - t0) / 100).max()):.2f} | rows summed p50 {float(rel[:, 2].median()):.2f} "
                      f"max {float(rel[:, 2].max()):.2f} | stores p50 {float(rel[:, 3].median()):.2f} max "
                      f"{float(rel[:, 3].max()):.2f}")
        s = w[off:off + 8 * 8 * 64].view(torch.int64).view(64, 8).cpu().double()
        live = s[:, 7] != 0
        if not live.any():
            continue
        s = s[s[:, 4] != 0]
        rel = (s[:, 4:] - s[:, :1]) / 100.0
        t0 = float(s[:, 0].min())
        print(f"hot wgs {len(s)} updating {int(live.sum())}: start p50/max {float(((s[:, 0] - t0) / 100).median()):.2f}/"
              f"{float(((s[:, 0] - t0) / 100).max()):.2f} | " + " | ".join(
                  f"s{k + 4} p50 {float(rel[:, k][rel[:, k] > 0].median()):.2f} max {float(rel[:, k].max()):.2f}"
                  for k in range(4) if (rel[:, k] > 0).any()))
