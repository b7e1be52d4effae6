"""World size 2 over gloo: sharding + the gather of encoded shards reproduce the single-process
encoding byte for byte.  On the CPU the shards are encoded by the oracle; the GPU variant encodes
each rank's shard with the HIP kernels (both ranks on cuda:0) and gathers over gloo.  The RCCL
gather itself (sbe_gather_encoded) is tested on one rank in test_gpu_config5.py; the 8-GPU run is
the driver's (bench.py's config5 leg)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pytest

import sbe_testlib as T


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import shard
    arena, L, ts = T.var_orders(n, seed=31)
    starts = np.concatenate([[0], np.cumsum(L.sum(1).astype(np.int64))])
    lo, hi = shard.shard_range(n, world, rank)
    a_r = arena[starts[lo]: starts[hi]]
    out, off, _ = T.oracle_encode(a_r, L[lo:hi], ts[lo:hi])
    res = shard.gather_encoded(torch.from_numpy(out.copy()), torch.from_numpy(off.view(np.int64).copy()), hi - lo, root=0)
    if rank == 0:
        q.put((res[0].numpy().tobytes(), res[1].numpy().tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    import shard
    for n in (0, 1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            r = [shard.shard_range(n, world, k) for k in range(world)]
            assert r[0][0] == 0 and r[-1][1] == n and all(r[k][1] == r[k + 1][0] for k in range(world - 1))


def test_gather_world2_matches_single_process():
    n, world = 3001, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    stream, offsets = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    arena, L, ts = T.var_orders(n, seed=31)
    eo, eoff, _ = T.oracle_encode(arena, L, ts)
    assert stream == bytes(eo)
    assert offsets == [int(x) for x in eoff]


def _worker_hip(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import shard
    import sbecodec
    arena, L, ts = T.var_orders(n, seed=37)
    starts = np.concatenate([[0], np.cumsum(L.sum(1).astype(np.int64))])
    lo, hi = shard.shard_range(n, world, rank)
    m = hi - lo
    a = torch.from_numpy(np.ascontiguousarray(arena[starts[lo]: starts[hi]])).cuda()
    enc = sbecodec.encode_topic_batch(a, torch.from_numpy(np.ascontiguousarray(L[lo:hi]).view(np.int32)).cuda(),
                                      torch.from_numpy(np.ascontiguousarray(ts[lo:hi]).view(np.int64)).cuda())
    torch.cuda.synchronize()
    off = enc.out_off[: m + 1].cpu()
    res = shard.gather_encoded(enc.out[: int(off[m])].cpu(), off, m, root=0)
    if rank == 0:
        q.put((res[0].numpy().tobytes(), res[1].numpy().tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_gather_world2_hip_shards():
    """Both ranks encode their shard on the GPU (HIP pack kernel), the gather runs over gloo."""
    n, world = 20011, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_hip, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    stream, offsets = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    arena, L, ts = T.var_orders(n, seed=37)
    eo, eoff, _ = T.oracle_encode(arena, L, ts)
    assert stream == bytes(eo)
    assert offsets == [int(x) for x in eoff]
