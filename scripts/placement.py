"""Pack-kernel time against buffer placement, in one process: the fixed-256 headline encode with its
input arena and output stream carved at different offsets of one large allocation (diagnosis of
the box-to-box / process-to-process spread of the pack kernel).  Prints one line per
placement: arena offset, output offset, median pack time from the library's HIP-event ring.
Usage: python scripts/placement.py [--steps K]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "aeron-cluster-client-cpp_amd"), os.path.join(ROOT, "tests")]
import sbe_testlib as T  # noqa: E402
import sbecodec  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=40)
args = ap.parse_args()

sbecodec.require_device()
dev = torch.device("cuda:0")
n = 1_000_000
arena_h, L, ts = T.fixed256_orders(n)
Ld = torch.from_numpy(L.view(np.int32)).to(dev)
tsd = torch.from_numpy(ts.view(np.int64)).to(dev)
A = arena_h.size
O = 256 * n
MB = 1 << 20
pool = torch.empty(A + O + 64 * MB, dtype=torch.uint8, device=dev)
src = torch.from_numpy(arena_h).to(dev)
oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
st = torch.empty(n, dtype=torch.uint8, device=dev)
ws = sbecodec.alloc_workspace(n, dev)
sbecodec.profile_enable(1)


def run(a_off, o_off):
    arena = pool[a_off:a_off + A]
    arena.copy_(src)
    out = pool[o_off:o_off + O + 16]
    for _ in range(10):
        sbecodec.encode_topic_batch(arena, Ld, tsd, out=out, out_off=oo, status=st, workspace=ws)
    torch.cuda.synchronize()
    sbecodec.profile_read(0)
    for _ in range(args.steps):
        sbecodec.encode_topic_batch(arena, Ld, tsd, out=out, out_off=oo, status=st, workspace=ws)
    torch.cuda.synchronize()
    ms = sorted(sbecodec.profile_read(0))
    return 1e3 * ms[len(ms) // 2]


K4 = 4096
configs = [(0, A + 32 * MB)]
for d in (0, 16, 64, 256, 1024, 4 * K4, 16 * K4, 64 * K4, 512 * K4):
    configs.append((0, A + 32 * MB + d))
for d in (K4, 16 * K4, 256 * K4):
    configs.append((d, A + 32 * MB))
configs.append((O + 32 * MB, 0))  # output below the input
configs.append((0, A + 32 * MB))  # the first placement again
for a_off, o_off in configs:
    print(f"arena@{a_off:>12d} out@{o_off:>12d} (rel {o_off - a_off:>12d})  pack {run(a_off, o_off):7.2f} us", flush=True)
