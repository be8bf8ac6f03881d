"""EXPERIMENT: per-workgroup start / end (wave 0, s_memrealtime, 100 MHz) of the ring's tail launch
(tower_tail_kernel: next-batch insert, tiles, bias/loss, hot and list roles), and T3's phases, at
the north-star shape (IDS=zipf: Zipf-skewed ids; GRAPH=1: the last tail of an 8-step graph replay). Times in us from each launch's first workgroup start; per role: start p50 / max, end p50 /
max."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["TT_RING_STAMPS"] = "1"
import torch  # noqa: E402

from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402

dev = torch.device("cuda:0")
N = [50_000_000, 100_000_000]
B = 8192
st = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, dev)
g = torch.Generator(device=dev).manual_seed(1)


def ids(n):
    if os.environ.get("IDS", "uniform") == "uniform":
        return torch.randint(0, n, (B,), generator=g, device=dev)
    # Zipf-like (s ~ 1.05) over permuted ranks, as bench.py --ids zipf
    u01 = torch.rand(B, generator=g, device=dev, dtype=torch.float64)
    r = torch.floor(torch.exp(u01 * torch.log(torch.tensor(float(n), device=dev, dtype=torch.float64))))
    return (r.to(torch.int64) * 2654435761) % n


batches = [([ids(n) for n in N], torch.randint(0, 2, (B,), generator=g, device=dev, dtype=torch.int32))
           for _ in range(64)]
st.capture_ring(batches, steps_per_graph=8)
nwg = B // 32
off = st.towers.nbytes - (((max(2 * nwg, 1024) * 8 + nwg * 16 * 9) * 8 + 255) // 256 * 256)
base = st.towers.ws[off:off + 8192 * 8].view(torch.int64)
ntile, nbias = 6 * 32, (2 * (128 + 64) + 1 + 3) // 4
roles_t2 = [("tiles", 0, ntile), ("bias", ntile, ntile + nbias), ("insert", ntile + nbias, 1024)]
dd_inl = int(os.environ.get("DD_INL", "0"))


def show(name, seg, roles):
    s = seg.view(-1, 2).cpu().double()
    used = int((s[:, 0] != 0).sum())
    s = s[:used]
    t0 = s[s[:, 0] != 0, 0].min()  # workgroups that returned before stamping hold 0
    rel = (s - t0) / 100.0
    out = [f"{name} grid {used} end max {float(rel[:, 1].max()):.2f}"]
    for rn, a, b in roles:
        r = rel[a:min(b, used)]
        if len(r):
            out.append(f"{rn}[{a}:{min(b, used)}] start {float(r[:, 0].median()):.2f}/{float(r[:, 0].max()):.2f} "
                       f"end {float(r[:, 1].median()):.2f}/{float(r[:, 1].max()):.2f}")
    print(" | ".join(out))


for it in range(6):
    base[4096:].zero_()
    if os.environ.get("GRAPH") == "1":  # the last tail of an 8-step graph replay
        st.run(8)
    else:
        st.run_eager(1)
    torch.cuda.synchronize()
    if it < 2:
        continue
    if st.ring_tail:
        n_ins, dd = 64, int(os.environ.get("K3_DD", "576"))
        show("tail", base[4096:6144], [("insert", 0, n_ins), ("tiles", n_ins, n_ins + ntile),
                                       ("bias", n_ins + ntile, n_ins + ntile + nbias),
                                       ("hot", n_ins + ntile + nbias, n_ins + ntile + nbias + 64),
                                       ("slots", n_ins + ntile + nbias + 64, n_ins + ntile + nbias + dd)])
        continue
    show("T2", base[4096:6144], roles_t2)
    k3 = base[6144:8192]
    used = int((k3.view(1024, 2)[:, 0] != 0).sum())
    dd = int(os.environ.get("K3_DD", "0"))
    show("K3", k3, [("resolver", 0, 32), ("rows", 32, 32 + dd), ("t3", 32 + dd, used)] if dd else
         [("resolver", 0, 32)] + [(f"wg{a}", a, a + 64) for a in range(32, used, 64)])

# T3 (tower_update_kernel) phases of the last step: 0 start, 1 gradient summed, 2 stores issued
if st.ring_tail:
    base[6144:].zero_()
    st.run_eager(1)
    torch.cuda.synchronize()
    t3 = base[6144:8192].view(512, 4).cpu().double()
    used = int((t3[:, 0] != 0).sum())
    t3 = t3[:used]
    rel = (t3[:, :3] - t3[:, 0].min()) / 100.0
    print(f"T3 grid {used}: start p50 {float(rel[:, 0].median()):.2f} max {float(rel[:, 0].max()):.2f} | "
          f"grad p50 {float(rel[:, 1].median()):.2f} max {float(rel[:, 1].max()):.2f} | "
          f"stores p50 {float(rel[:, 2].median()):.2f} max {float(rel[:, 2].max()):.2f}")
