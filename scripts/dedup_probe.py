"""Device time of the single-hot backward, old (hash/scan/scatter + narrow/hot) vs new (insert +
update), north-star shapes; graph-timed back-to-back launches (HIP events on the replay stream)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from two_tower_recommender_model_amd import ops
from bench import time_kernel

dev = torch.device("cuda:0")
N = [50_000_000, 100_000_000]
B, D = 8192, 128
for ids in ("uniform", "zipf"):
    ts = ops.TableSet(N, [D, D], [0, 1], dev)
    ts.init_uniform_(torch.Generator(device=dev).manual_seed(0))
    g = torch.Generator(device=dev).manual_seed(1)
    if ids == "uniform":
        cols = [torch.randint(0, n, (B,), generator=g, device=dev) for n in N]
    else:
        cols = []
        for n in N:
            u = torch.rand(B, generator=g, device=dev, dtype=torch.float64)
            r = torch.floor(torch.exp(u * torch.log(torch.tensor(float(n), device=dev, dtype=torch.float64))))
            cols.append((r.to(torch.int64) * 2654435761) % n)
    gout = torch.randn(B, 2 * D, device=dev)
    ts.ensure_bwd_workspace(2 * B)
    ts.ensure_dedup_workspace(2 * B)
    def old():
        ts.bwd_prepare_cols(cols, N)
        ts.bwd_rowwise_adagrad(gout, None, B, 0.0, 1e-10)
    def new():
        ts.dedup_insert_cols(cols, N)
        ts.dedup_rowwise_adagrad(gout, B, 0.0, 1e-10)
    t_old = time_kernel(old, 20)
    t_new = time_kernel(new, 20)
    t_ins = None
    print(f"{ids}: old prepare+update {t_old*1e3:.2f} us, new insert+update {t_new*1e3:.2f} us", flush=True)
