"""Diagnostic: time the tower kernels (T1, T2, T3) alone at the north-star shape.
Not part of the product or the tests."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from two_tower_recommender_model_amd import ops  # noqa: E402

B = int(os.environ.get("T1_B", 8192))
dev = torch.device("cuda:0")
in_dims, widths, in_cols = [128, 128], [128, 64], [0, 128]
ft = ops.FusedTowers(in_dims, widths, in_cols, B, dev)
params = torch.randn(ft.num_params, device=dev) * 0.05
pooled = torch.randn(B, 256, device=dev)
gpooled = torch.empty_like(pooled)
labels = torch.randint(0, 2, (B,), device=dev, dtype=torch.int32)
logits = torch.empty(B, device=dev)
loss = torch.empty(1, device=dev)
ft.update(params, do_adam=False)
torch.cuda.synchronize()

def timed(fn, n=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1000


print(f"T1 fwd_bwd: {timed(lambda: ft.fwd_bwd(pooled, gpooled, params, labels, logits)):.2f} us/launch")
print(f"T2 wgrad  : {timed(lambda: ft.wgrad(loss)):.2f} us/launch")
print(f"T3 update : {timed(lambda: ft.update(params, do_adam=False)):.2f} us/launch", flush=True)
