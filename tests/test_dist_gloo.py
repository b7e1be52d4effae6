"""CPU, world_size 2 (gloo): sharding + gatherv of encoded shards reproduce the single-process
encoding byte for byte.  The shards are encoded by the oracle here (no GPU); on the GPU box the
same shard.gather_encoded runs over RCCL on device tensors (bench.py --gather)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

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
