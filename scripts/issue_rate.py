"""Host issue cost of bench.py's step (encode + decode calls through the ctypes binding), without
GPU synchronisation: if it approaches the GPU time per step, the timed loop is host-bound."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "aeron-cluster-client-cpp_amd"), os.path.join(ROOT, "tests")]
import sbe_testlib as T  # noqa: E402
import sbecodec  # noqa: E402

n = 1_000_000
dev = torch.device("cuda:0")
arena, L, ts = T.fixed256_orders(n)
a, l, t = (torch.from_numpy(arena).to(dev), torch.from_numpy(L.view(np.int32)).to(dev),
           torch.from_numpy(ts.view(np.int64)).to(dev))
out = torch.empty(sbecodec.output_bound(n, arena.size), dtype=torch.uint8, device=dev)
off = torch.empty(n + 1, dtype=torch.int64, device=dev)
st = torch.empty(n, dtype=torch.uint8, device=dev)
ws = sbecodec.alloc_workspace(n, dev)
dec = sbecodec.alloc_decoded(n, dev)
seq = torch.zeros(n, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream()


def step():
    sbecodec.encode_topic_batch(a, l, t, out=out, out_off=off, status=st, workspace=ws, stream=s)
    sbecodec.decode_batch(out, off, mode=sbecodec.DEC_PARSE_MESSAGE, out=dec, stream=s, seq=seq)


for _ in range(5):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(200):
    step()
issue = (time.perf_counter() - t0) / 200
torch.cuda.synchronize()
gpu = (time.perf_counter() - t0) / 200
print(f"host issue {issue * 1e6:.1f} us/step, wall incl. GPU {gpu * 1e6:.1f} us/step")
