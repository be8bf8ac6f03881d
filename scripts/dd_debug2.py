"""DEBUG: T1 deferred inserts vs the resolver, recycled garbage memory."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep
dev = torch.device("cuda:0")
junk = torch.randint(0, 255, (1 << 29,), dtype=torch.uint8, device=dev)
del junk
B, D, N = 1024, 128, [20000, 30000]
st = FusedTwoTowerStep(N, [D, D], [0], [1], [128, 64], B, dev, kjt_mode="cols", seed=5, materialize_pooled=True, dedup="single")
g = torch.Generator().manual_seed(1)
L = 2 * B
cap = 1024
while cap < 4 * L:
    cap <<= 1
al = lambda x: (x + 255) // 256 * 256  # noqa: E731
o_lkey = al(cap * 64); o_hot = o_lkey + al(L * 8); o_ctr = o_hot + al((L // 15 + 1) * 4); o_claim = o_ctr + 256
o_ovf = o_claim + al(4 * L); G = (L + 63) // 64
ws = st.tables._dd_ws
tabs = [st.tables.table_view(0), st.tables.table_view(1)]
for s in range(3):
    cols = [torch.randint(0, 2 * n, (B,), generator=g) for n in N]
    lab = torch.randint(0, 2, (B,), generator=g).to(torch.int32)
    st.load_batch([c.to(dev) for c in cols], lab.to(dev))
    st.towers.fwd_bwd_gather(st.cols, st.num_embeddings, tabs, st.gpooled, st.params, st.labels, st.logits,
                             dedup=st.tables, dedup_tables=(0, 1))
    torch.cuda.synchronize()
    claim = ws[o_claim:o_claim + 4 * L].view(torch.int32).cpu()
    ovf = ws[o_ovf:o_ovf + 16 * 64 * G].view(torch.int64).view(G, 64, 2).cpu()
    dk = ovf[:, :, 0] != -1
    deferred = sorted((ovf[:, :, 1][dk] & 0xffffffff).tolist())
    neg = (claim == -1).nonzero().flatten().tolist()
    print("step", s, "deferred", len(deferred), "claim -1", len(neg), "same set", deferred == neg, flush=True)
    st.tables.dedup_resolve()
    torch.cuda.synchronize()
    claim2 = ws[o_claim:o_claim + 4 * L].view(torch.int32).cpu()
    left = int((ws[o_ovf:o_ovf + 16 * 64 * G].view(torch.int64).view(G, 64, 2)[:, :, 0] != -1).sum())
    print("   after resolve: claims -1:", int((claim2 == -1).sum()), "ovf left", left, flush=True)
    st.tables.dedup_rowwise_adagrad(st.gpooled, B, 0.01, 1e-10)
    torch.cuda.synchronize()
