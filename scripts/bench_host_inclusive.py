"""Host-inclusive rate: the path as the reference sees it starts and ends in host
memory (Aeron /dev/shm buffers).  Times H2D(input) → encode → decode → D2H(stream + descriptors)
with pinned buffers, double-buffered over two streams.  Reported in DESIGN.md, never as `value`."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "aeron-cluster-client-cpp_amd"), os.path.join(ROOT, "tests")]
import sbe_testlib as T  # noqa: E402
import sbecodec  # noqa: E402


def main(n=1_000_000, iters=10):
    sbecodec.require_device()
    dev = torch.device("cuda:0")
    arena, L, ts = T.fixed256_orders(n)
    h_arena = torch.from_numpy(arena).pin_memory()
    h_len = torch.from_numpy(L.view(np.int32)).pin_memory()
    h_ts = torch.from_numpy(ts.view(np.int64)).pin_memory()
    cap = sbecodec.output_bound(n, arena.size)
    streams = [torch.cuda.Stream() for _ in range(2)]
    bufs = []
    for s in streams:
        with torch.cuda.stream(s):
            bufs.append(dict(
                a=torch.empty_like(h_arena, device=dev), l=torch.empty_like(h_len, device=dev),
                t=torch.empty_like(h_ts, device=dev), out=torch.empty(cap, dtype=torch.uint8, device=dev),
                off=torch.empty(n + 1, dtype=torch.int64, device=dev), st=torch.empty(n, dtype=torch.uint8, device=dev),
                ws=sbecodec.alloc_workspace(n, dev, s), dec=sbecodec.alloc_decoded(n, dev),
                h_out=torch.empty(cap, dtype=torch.uint8).pin_memory(),
                h_dec=[torch.empty_like(x, device="cpu").pin_memory() for x in (None,) if False]))
    h_desc = [{k: torch.empty(getattr(b["dec"], k).shape, dtype=getattr(b["dec"], k).dtype).pin_memory()
               for k in ("status", "flags", "hdr", "ts", "view_off", "view_len")} for b in bufs]

    def one(i):
        s, b, hd = streams[i % 2], bufs[i % 2], h_desc[i % 2]
        with torch.cuda.stream(s):
            b["a"].copy_(h_arena, non_blocking=True)
            b["l"].copy_(h_len, non_blocking=True)
            b["t"].copy_(h_ts, non_blocking=True)
            sbecodec.encode_topic_batch(b["a"], b["l"], b["t"], out=b["out"], out_off=b["off"], status=b["st"],
                                        workspace=b["ws"], stream=s)
            sbecodec.decode_batch(b["out"], b["off"], out=b["dec"], stream=s)
            b["h_out"][: 256 * n].copy_(b["out"][: 256 * n], non_blocking=True)
            for k, v in hd.items():
                v.copy_(getattr(b["dec"], k), non_blocking=True)

    for i in range(2):
        one(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(iters):
        one(i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"metric": "host-inclusive encode+decode rec/s (pinned H2D + kernels + D2H)",
                      "records": n, "iters": iters, "value": n * iters / el,
                      "h2d_bytes_per_rec": 250, "d2h_bytes_per_rec": 256 + 58}))


if __name__ == "__main__":
    main()
