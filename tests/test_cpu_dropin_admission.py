"""Host logic of the N > 1 drop-in's agreed admission (dropin.FusedShardedDropin, no GPU): the
admission vector a rank builds from its shape checks and tt_kjt_admit's counts, and the decision
taken on the MAX over the ranks — every rank must take the same path for a batch."""
import types

import numpy as np
import torch

from two_tower_recommender_model_amd import dropin
from two_tower_recommender_model_amd.dropin import (A_B, A_DEST, A_DT, A_ERR, A_MULTI, A_NEGB, A_NEGDT, A_NNZ, A_OVER,
                                                    A_REJECT, A_SEG, FusedShardedDropin)


def _fd(W=2, sharding=("row_wise", "row_wise"), mode=None, step=None):
    fd = object.__new__(FusedShardedDropin)
    fd.W, fd.sharding, fd.mode, fd.step = W, list(sharding), mode, step
    fd.id_dtype = torch.int64
    return fd


def _batch(B, nnz, dtype=torch.int64):
    kjt = types.SimpleNamespace(stride=lambda: B, values=lambda: torch.zeros(nnz, dtype=dtype))
    return types.SimpleNamespace(sparse_features=kjt)


def _counts(W, multi, err, cnt):
    c = np.zeros(2 + 2 * W, dtype=np.int32)
    c[0], c[1] = multi, err
    c[2:] = np.asarray(cnt, dtype=np.int32).reshape(-1)
    return torch.from_numpy(c)


def test_vector_from_counts_and_caps():
    W = 2
    step = types.SimpleNamespace(caps_f=[300, 300], cap=900, B=512)
    fd = _fd(W, mode="pipelined", step=step)
    # cnt[d][f]: owner 0 gets 301 of feature 1 -> over its capacity 300
    a = fd._vector(True, _batch(512, 1000), _counts(W, 0, 0, [[250, 301], [240, 209]])).numpy()
    assert a[A_REJECT] == 0 and a[A_B] == 512 and a[A_NEGB] == -512 and a[A_DT] == 1 and a[A_NEGDT] == -1
    assert a[A_SEG] == 301 and a[A_DEST] == 551 and a[A_NNZ] == 1000 and a[A_OVER] == 1 and a[A_MULTI] == 0
    fd.mode = "kjt"
    a = fd._vector(True, _batch(512, 1000), _counts(W, 1, 0, [[250, 301], [240, 209]])).numpy()
    assert a[A_OVER] == 0 and a[A_MULTI] == 1  # 551 ids for owner 0 <= cap 900; bags of several ids allowed
    # table-wise features never count toward the segment capacities (their owner segment holds B)
    fd = _fd(W, sharding=("table_wise", "row_wise"), mode="pipelined", step=step)
    a = fd._vector(True, _batch(512, 1000), _counts(W, 0, 0, [[512, 10], [0, 20]])).numpy()
    assert a[A_SEG] == 20 and a[A_OVER] == 0


def test_rejection_and_agreement():
    W = 2
    step = types.SimpleNamespace(caps_f=[300, 300], cap=900, B=512)
    fd = _fd(W, mode="pipelined", step=step)
    ok = fd._vector(True, _batch(512, 1000), _counts(W, 0, 0, [[100, 100], [100, 100]]))
    bad = fd._vector(False, _batch(512, 1000), None)
    assert bad.numpy()[A_REJECT] == 1
    ag = torch.maximum(ok, bad).numpy()  # what the MAX all-reduce gives every rank
    assert "shape" in fd._reason(ag)
    assert fd._reason(ok.numpy()) == ""
    # batch sizes differ across the ranks: B and -B do not agree after the MAX
    other = fd._vector(True, _batch(504, 1000), _counts(W, 0, 0, [[100, 100], [100, 100]]))
    assert "batch sizes" in fd._reason(torch.maximum(ok, other).numpy())
    # an int32 batch on one rank, int64 on the other
    i32 = fd._vector(True, _batch(512, 1000, torch.int32), _counts(W, 0, 0, [[100, 100], [100, 100]]))
    assert "dtypes" in fd._reason(torch.maximum(ok, i32).numpy())
    # one rank's bag of two ids sends the batch down the generic path on every rank (pipelined mode)
    multi = fd._vector(True, _batch(512, 1000), _counts(W, 1, 0, [[100, 100], [100, 100]]))
    assert "several ids" in fd._reason(torch.maximum(ok, multi).numpy())
    fd.mode = "kjt"
    assert fd._reason(torch.maximum(ok, multi).numpy()) == ""
    fd.mode = "pipelined"
    over = fd._vector(True, _batch(512, 1000), _counts(W, 0, 0, [[400, 100], [100, 100]]))
    assert "capacity" in fd._reason(torch.maximum(ok, over).numpy())
    err = fd._vector(True, _batch(512, 1000), _counts(W, 0, 2, [[100, 100], [100, 100]]))
    assert "outside" in fd._reason(torch.maximum(ok, err).numpy())
    assert err.numpy()[A_ERR] == 2


def test_first_batch_ignores_capacity_and_bag_length():
    """Before a step exists there is no capacity yet, and the first batch's bag lengths choose the
    mode (multi-hot: the KJT step) instead of rejecting it."""
    fd = _fd(2)
    v = fd._vector(True, _batch(512, 3000), _counts(2, 1, 0, [[700, 800], [750, 750]])).numpy()
    assert v[A_OVER] == 0 and v[A_MULTI] == 1
    assert fd._reason(v, first=True) == ""
    assert dropin.A_LEN >= A_NNZ + 1
