"""Practical HBM ceiling for the pack kernel's traffic shape: a device copy moving the same bytes
(read 250 MB, write 265 MB per 1 M fixed-256 records), timed with HIP events.  Reported in
DESIGN.md next to the 8 TB/s spec peak."""
import json

import torch


def main(nbytes_r=250_000_000, nbytes_w=265_000_000, iters=50):
    src = torch.empty(nbytes_r, dtype=torch.uint8, device="cuda")
    dst = torch.empty(nbytes_w, dtype=torch.uint8, device="cuda")
    src.fill_(1)
    n = min(nbytes_r, nbytes_w)
    for _ in range(5):
        dst[:n].copy_(src[:n])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        dst[:n].copy_(src[:n])
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    print(json.dumps({"what": "torch device copy", "bytes_read": n, "bytes_written": n, "ms": ms,
                      "GBps": 2 * n / (ms * 1e-3) / 1e9}))
    # a 2-D strided read + contiguous write, closer to a gather/scatter of 256-B rows
    a = torch.empty((1_000_000, 256), dtype=torch.uint8, device="cuda")
    b = torch.empty((1_000_000, 222), dtype=torch.uint8, device="cuda")
    for _ in range(5):
        a[:, :222].copy_(b)
    e0.record()
    for _ in range(iters):
        a[:, :222].copy_(b)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    print(json.dumps({"what": "torch copy of 222-B rows into 256-B rows", "ms": ms,
                      "GBps": (222 + 222) * 1_000_000 / (ms * 1e-3) / 1e9}))


if __name__ == "__main__":
    main()
