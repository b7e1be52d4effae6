"""Multi-GPU sharding of record batches and the gather of encoded shards.

Records are independent, so a batch shards by contiguous index ranges with no data-path
collective; the only exchange is the optional gather of the encoded byte streams to one rank
(what an ingress publisher on that rank would offer).  One process per GPU.

Two gathers, one protocol (an all-gather of the 8-byte shard sizes, then point-to-point sends
into the root's prefix offsets: RCCL has no gatherv):
  RcclGather      the product path: sbe_gather_encoded in libsbecodec.so (include/sbecodec.h),
                  RCCL over xGMI, the same entry point a C++ ingress publisher calls;
  gather_encoded  the same exchange over torch.distributed, for CPU tensors on the gloo backend
                  (tests/test_dist_gloo.py runs the sharded pipeline's host side with it).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Records [lo, hi) of `rank`: record i goes to rank ⌊i·world/n⌋."""
    return n * rank // world, n * (rank + 1) // world


class RcclGather:
    """sbe_gather_encoded over one RCCL communicator per rank, created collectively from a
    torch.distributed group (its id travels through the group; the data never does)."""

    def __init__(self, group=None):
        import sbecodec
        self._codec = sbecodec
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        box = [sbecodec.comm_unique_id() if self.rank == 0 else None]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        self.comm = sbecodec.Comm(self.world, self.rank, box[0])

    def gather(self, out, out_off, n: int, root: int = 0, dst=None, dst_off=None, stream=None):
        """Every rank's out[:out_off[n]] back to back on `root` (group rank), offsets rebased.
        Returns (stream, offsets, bytes, records) on the root, (None, None, bytes, records) elsewhere."""
        return self._codec.gather_encoded(self.comm, out, out_off, n, root=root, dst=dst, dst_off=dst_off,
                                          stream=stream)

    def gather_sized(self, sizes, out, out_off, root: int = 0, dst=None, dst_off=None, dst_capacity: int = 0,
                     dst_off_capacity: int = 0, stream=None):
        """The same for callers that know every rank's shard size (sizes = [(bytes, records)] per
        group rank, identical on every rank; fixed-size records, or a host size plan): no size
        all-gather and no host wait (sbe_gather_encoded_sized), so the next shard's encode can be
        enqueued while this one travels.  Every rank passes the root's capacities."""
        return self._codec.gather_encoded_sized(self.comm, sizes, out, out_off, root=root, dst=dst, dst_off=dst_off,
                                                dst_capacity=dst_capacity, dst_off_capacity=dst_off_capacity,
                                                stream=stream)

    def close(self):
        self.comm.close()


def gather_encoded(out: torch.Tensor, out_off: torch.Tensor, n: int, root: int = 0, group=None):
    """Gather every rank's encoded stream out[:out_off[n]] and its record offsets to `root` (a rank
    of `group`) over torch.distributed.

    Returns (stream uint8 [total], offsets int64 [N+1]) on root, None elsewhere.  out_off holds
    the n+1 local offsets (device or host tensor, as the backend requires)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)

    def peer(r):  # P2POp peers are global ranks
        return dist.get_global_rank(group, r) if group is not None else r

    dev = out.device
    local_bytes = out_off[n: n + 1].to(torch.int64).clone()
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    counts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, local_bytes, group=group)
    dist.all_gather(counts, torch.tensor([n], dtype=torch.int64, device=dev), group=group)
    sizes = torch.cat(sizes).tolist()  # one host synchronisation for all sizes
    counts = torch.cat(counts).tolist()
    if rank != root:
        ops = []
        if sizes[rank]:
            ops.append(dist.P2POp(dist.isend, out[: sizes[rank]].contiguous(), peer(root), group))
        ops.append(dist.P2POp(dist.isend, out_off[:n].to(torch.int64).contiguous(), peer(root), group))
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
            ops.append(dist.P2POp(dist.irecv, stream[base[r]: base[r] + sizes[r]], peer(r), group))
        buf = torch.empty(counts[r], dtype=torch.int64, device=dev)
        recv_off[r] = buf
        ops.append(dist.P2POp(dist.irecv, buf, peer(r), group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    for r, buf in recv_off.items():
        offsets[rbase[r]: rbase[r] + counts[r]].copy_(buf + base[r])
    offsets[-1] = total
    return stream[:total], offsets
