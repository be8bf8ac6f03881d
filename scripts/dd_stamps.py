"""EXPERIMENT: per-phase wall time of the fused row-wise Adagrad's slot workgroups from
s_memrealtime stamps (100 MHz): 0 start, 1 slot + meta in, 2 gradient rows summed, 3 stores issued.
MODE=alone: T1 + T2 + the update launch on its own; MODE=step (default): the combined K2."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["TT_DD_STAMPS"] = "1"
import torch
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep

dev = torch.device("cuda:0")
N = [50_000_000, 100_000_000]; B = 8192
st = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, dev)
g = torch.Generator(device=dev).manual_seed(1)
st.load_batch([torch.randint(0, n, (B,), generator=g, device=dev) for n in N],
              torch.randint(0, 2, (B,), generator=g, device=dev, dtype=torch.int32))
tabs = [st.tables.table_view(0), st.tables.table_view(1)]
L = 2 * B
cap = 1024
while cap < 4 * L:
    cap <<= 1
al = lambda x: (x + 255) // 256 * 256  # noqa: E731
G = (L + 63) // 64
off = al(cap * 64) + al(L * 8) + al((L // 15 + 1) * 4) + al(16) + al(4 * L) + al(16 * 64 * G)
nwg = L // 32 + 32
ws = st.tables._dd_ws
mode = os.environ.get("MODE", "step")
for it in range(6):
    if mode == "alone":
        st.towers.fwd_bwd_gather(st.cols, st.num_embeddings, tabs, st.gpooled, st.params, st.labels, st.logits,
                                 dedup=st.tables, dedup_tables=(0, 1))
        st.towers.wgrad(st.loss)
        st.tables.dedup_resolve()
        st.tables.dedup_rowwise_adagrad(st.gpooled, B, st.lr_emb, st.eps)
    else:
        st.step()
    torch.cuda.synchronize()
    stm = ws[off:off + nwg * 64].view(torch.int64).view(nwg, 8).cpu().double()
    if it < 2:
        continue
    hot = 32
    s = stm[hot:]
    t0 = s[:, 0].min()
    rel = (s[:, :4] - t0) * 10 / 1000  # us
    q = lambda c, p: float(torch.quantile(rel[:, c], p))  # noqa: E731
    print(f"{mode} it{it}: start p50 {q(0, .5):.2f} p90 {q(0, .9):.2f} max {q(0, 1):.2f} | "
          f"slot-in {float((rel[:, 1] - rel[:, 0]).median()):.2f} | rows {float((rel[:, 2] - rel[:, 1]).median()):.2f} | "
          f"tail {float((rel[:, 3] - rel[:, 2]).median()):.2f} | end p50 {q(3, .5):.2f} max {q(3, 1):.2f}")
