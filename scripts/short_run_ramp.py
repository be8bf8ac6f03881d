"""Per-step time of consecutive short timed runs (20 steps each, synchronised on both sides) after
a 5-step warmup at the north-star shape: whether the first timed run after capture pays a ramp."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
N, B = [50_000_000, 100_000_000], 8192
st = FusedTwoTowerStep(N, [128, 128], [0], [1], [128, 64], B, dev, lr_emb=0.01, lr_dense=0.01, seed=0)
batches = bench.synth_batches(N[0], N[1], B, 64, dev, "uniform", seed=1)
st.capture_ring(batches, steps_per_graph=8)
st.align_ring(20, after=5)
st.run(5)
torch.cuda.synchronize()
out = []
for rep in range(6):
    t0 = time.perf_counter()
    st.run(20 if rep < 5 else 40)
    torch.cuda.synchronize()
    out.append((time.perf_counter() - t0) / (20 if rep < 5 else 40) * 1e6)
print("us/step of consecutive timed runs (20, 20, 20, 20, 20, 40 steps):", [round(x, 2) for x in out])
