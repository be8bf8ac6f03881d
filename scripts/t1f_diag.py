"""EXPERIMENT: which part of the ring diverges from the classic step — the 64-wide row-owned T1 or
the T3 folded into T1 — after k steps (eager without intermediate flushes, or graphs), D in {64, 128}."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tests.test_gpu_ring import _batches  # noqa: E402
from two_tower_recommender_model_amd.fused import FusedTwoTowerStep  # noqa: E402

dev = torch.device("cuda:0")
N, B = [30_000, 50_000], 2048
d = lambda x, y: float((x - y).abs().max())  # noqa: E731
for D in (128, 64):
    batches = _batches(N, B, 6, seed=D, device=dev)
    b = FusedTwoTowerStep(N, [D, D], [0], [1], [128, 64], B, dev, seed=2)
    ref = []
    for s in range(4):
        b.load_batch(*batches[s])
        b.step()
        torch.cuda.synchronize()
        ref.append([t.clone() for t in (b.tables.weights, b.tables.state, b.params, b.exp_avg, b.logits, b.grads)]
                   + [float(b.loss)])
    del b
    for mode in ("eager", "graph"):
        for fuse in (False, True):
            for k in (1, 2, 3, 4):
                a = FusedTwoTowerStep(N, [D, D], [0], [1], [128, 64], B, dev, seed=2)
                if not fuse:
                    a._t1f = False
                a.capture_ring(batches, steps_per_graph=2)
                if mode == "eager":
                    a.run_eager(k, flush=False)
                    a.flush()
                else:
                    a.run(k)
                torch.cuda.synchronize()
                r = ref[k - 1]
                got = [a.tables.weights, a.tables.state, a.params, a.exp_avg, a.logits, a.grads]
                diffs = " ".join(f"{n} {d(x, y):.1e}" for n, x, y in zip(("tab", "st", "prm", "m", "logit", "gp"), got, r))
                print(f"D={D} {mode} fuse={fuse} k={k}: {diffs} loss {abs(float(a.loss) - r[6]):.1e} "
                      f"timeouts={a.fuse_timeouts()}", flush=True)
                del a
                torch.cuda.empty_cache()
