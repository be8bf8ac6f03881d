"""CPU: the sharded-step routing restatement (oracle.ref.shard_route) agrees with the pinned KJT
restatements it composes — transform_to_torchrec_batch (kjt_build) + fbgemm block_bucketize
(row-wise) — segment by segment, in bag order; and the capacity rule of the fused sharded step."""
import numpy as np
import pytest

from oracle import ref


@pytest.mark.parametrize("W", [1, 2, 3, 8])
def test_shard_route_matches_block_bucketize(W):
    rng = np.random.default_rng(W)
    B, N = 300, [1000, 777]
    cols = [rng.integers(-2 * n, 3 * n, B) for n in N]
    for c in cols:
        c[rng.random(B) < 0.1] = 0
    bs = [-(-n // W) for n in N]
    C = B
    send, pos, ovf = ref.shard_route(cols, N, bs, [0, 0], W, C)
    assert not ovf
    v, l, o = ref.kjt_build(cols, N)
    nl, nv = ref.block_bucketize(l, v.astype(np.int64), 2, B, bs, W)
    # bucket-major [W][F][B] lengths/values == segments (d, f) in bag order
    no = ref.complete_cumsum(nl)
    for d in range(W):
        for f in range(2):
            i0 = (d * 2 + f) * B
            want = nv[no[i0]:no[i0 + B]]
            n = int(send[d, f])
            got = send[d, 2 + f * C:2 + f * C + n] & ((1 << 40) - 1)
            np.testing.assert_array_equal(got, want)
            assert np.all((send[d, 2 + f * C:2 + f * C + n] >> 40) == f)
    # pos points every kept lookup at its own key
    for f in range(2):
        for b in range(B):
            p = pos[f * B + b]
            if cols[f][b] == 0:
                assert p == -1
                continue
            d, rest = divmod(int(p), 2 * C)
            ff, k = divmod(rest, C)
            assert ff == f
            row = int(np.mod(cols[f][b], N[f]))
            assert send[d, 2 + f * C + k] == (f << 40) | (row - d * bs[f])


def test_shard_route_table_wise_and_overflow():
    B, N = 64, [50, 60]
    cols = [np.arange(1, B + 1), np.arange(1, B + 1) * 3]
    send, pos, ovf = ref.shard_route(cols, N, [0, 0], [1, 0], 2, 40)
    assert ovf  # 64 lookups of each table land in one segment of capacity 40
    assert send[1, 0] == 40 and send[0, 1] == 40 and send[0, 0] == 0 and send[1, 1] == 0
    assert (pos[:B] >= 0).sum() == 40 and (pos[B:] >= 0).sum() == 40


def test_default_capacity():
    from two_tower_recommender_model_amd.sharded import default_capacity

    assert default_capacity(8192, 1) == 8192
    c = default_capacity(8192, 8)
    # mean 1024, sd ~30 for uniform ids: far above mean + 6 sd, far below B
    assert 1024 + 6 * 30 < c < 2048 and c % 8 == 0
