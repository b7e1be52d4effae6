"""Multi-GPU sharding of record batches and the RCCL gather of encoded shards.

Records are independent, so a batch shards by contiguous index ranges with no data-path
collective; the only exchange is the optional gather of the encoded byte streams to one rank
(what an ingress publisher on that rank would offer).  One process per GPU; on ROCm the
torch.distributed "nccl" backend is RCCL over xGMI.  The gather is a gatherv: one all_gather of
the 8-byte shard sizes, then grouped point-to-point sends into the root's prefix offsets (RCCL has
no gatherv).  The same code runs on gloo with CPU tensors (tests/test_dist_gloo.py).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Records [lo, hi) of `rank`: record i goes to rank ⌊i·world/n⌋."""
    return n * rank // world, n * (rank + 1) // world


def gather_encoded(out: torch.Tensor, out_off: torch.Tensor, n: int, root: int = 0, group=None):
    """Gather every rank's encoded stream out[:out_off[n]] and its record offsets to `root`.

    Returns (stream uint8 [total], offsets int64 [N+1]) on root, None elsewhere.  out_off holds
    the n+1 local offsets (device or host tensor, as the backend requires)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = out.device
    local_bytes = out_off[n: n + 1].to(torch.int64).clone()
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    counts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, local_bytes, group=group)
    dist.all_gather(counts, torch.tensor([n], dtype=torch.int64, device=dev), group=group)
    sizes = [int(s.item()) for s in sizes]
    counts = [int(c.item()) for c in counts]
    if rank != root:
        ops = []
        if sizes[rank]:
            ops.append(dist.P2POp(dist.isend, out[: sizes[rank]].contiguous(), root, group))
        ops.append(dist.P2POp(dist.isend, out_off[:n].to(torch.int64).contiguous(), root, group))
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        return None
    total = sum(sizes)
    stream = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    offsets = torch.empty(sum(counts) + 1, dtype=torch.int64, device=dev)
    base = [sum(sizes[:r]) for r in range(world)]
    rbase = [sum(counts[:r]) for r in range(world)]
    ops, recv_off = [], {}
    for r in range(world):
        if r == root:
            stream[base[r]: base[r] + sizes[r]].copy_(out[: sizes[r]])
            offsets[rbase[r]: rbase[r] + counts[r]].copy_(out_off[:n].to(torch.int64))
            continue
        if sizes[r]:
            ops.append(dist.P2POp(dist.irecv, stream[base[r]: base[r] + sizes[r]], r, group))
        buf = torch.empty(counts[r], dtype=torch.int64, device=dev)
        recv_off[r] = buf
        ops.append(dist.P2POp(dist.irecv, buf, r, group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    for r, buf in recv_off.items():
        offsets[rbase[r]: rbase[r] + counts[r]].copy_(buf + base[r])
    offsets[-1] = total
    return stream[:total], offsets
