"""The seeded synthetic workloads themselves: the device-side generators that the
bench and the large GPU tests use produce the same bytes as the numpy generators the oracle tests
use, and config-5 shards concatenate to the single batch (CPU torch; the ops are device-agnostic)."""
import numpy as np
import torch

import sbe_testlib as T


def test_var_orders_torch_matches_numpy():
    for n, seed in ((1, 3), (777, 0x5EED0004), (20000, 31)):
        a, L, ts = T.var_orders(n, seed=seed)
        at, Lt, tt = T.var_orders_t(n, "cpu", seed=seed, chunk=4096)
        assert np.array_equal(a, at.numpy())
        assert np.array_equal(L.view(np.int32), Lt.numpy())
        assert np.array_equal(ts.view(np.int64), tt.numpy())


def test_var_orders_shape():
    a, L, ts = T.var_orders(5000, seed=9)
    Ls = L.astype(np.int64)
    assert a.size == Ls.sum()
    assert ((Ls[:, 3] >= 32) & (Ls[:, 3] <= 480)).all() and ((Ls[:, 4] >= 16) & (Ls[:, 4] <= 64)).all()
    assert (Ls[:, 2] == 29).all()
    assert not np.any(a == ord("\\"))


def test_config5_shards_concatenate():
    N = 5000
    whole = T.config5_shard(0, N, "cpu", chunk=1024)
    parts = [T.config5_shard(lo, hi, "cpu", chunk=700) for lo, hi in ((0, 1234), (1234, 4000), (4000, N))]
    for k in range(3):
        assert torch.equal(whole[k], torch.cat([p[k] for p in parts]))
