"""Diagnosis: kernel time of back-to-back encode-only and decode-only launches at several sizes
(is the per-launch overhead a property of the kernel or of the encode→decode hand-over?), and
the host-side cost of one encode / decode call through the Python binding."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "aeron-cluster-client-cpp_amd"), os.path.join(ROOT, "tests")]
import sbe_testlib as T  # noqa: E402
import sbecodec  # noqa: E402

sbecodec.require_device()
dev = torch.device("cuda:0")
for n in (1_000_000, 2_000_000, 4_000_000):
    arena, L, ts = T.fixed256_orders(n)
    a = torch.from_numpy(arena).to(dev)
    l = torch.from_numpy(L.view(np.int32)).to(dev)
    t = torch.from_numpy(ts.view(np.int64)).to(dev)
    ws = sbecodec.alloc_workspace(n, dev)
    enc = sbecodec.encode_topic_batch(a, l, t, workspace=ws)
    dec = sbecodec.decode_batch(enc.out, enc.out_off)
    torch.cuda.synchronize()
    res = {}
    for what in ("enc", "dec", "pair"):
        sbecodec.profile_enable(True)
        for _ in range(20):
            if what in ("enc", "pair"):
                sbecodec.encode_topic_batch(a, l, t, out=enc.out, out_off=enc.out_off, status=enc.status, workspace=ws)
            if what in ("dec", "pair"):
                sbecodec.decode_batch(enc.out, enc.out_off, out=dec)
        torch.cuda.synchronize()
        pk = sbecodec.profile_read(sbecodec.PROF_PACK)
        dk = sbecodec.profile_read(sbecodec.PROF_DECODE)
        sbecodec.profile_enable(False)
        res[what] = (np.median(pk) * 1e3 if pk else 0.0, np.median(dk) * 1e3 if dk else 0.0)
    # host cost per call (the queue absorbs the launches; 50 calls stay well inside it)
    torch.cuda.synchronize()
    h0 = time.perf_counter()
    for _ in range(50):
        sbecodec.encode_topic_batch(a, l, t, out=enc.out, out_off=enc.out_off, status=enc.status, workspace=ws)
    h1 = time.perf_counter()
    for _ in range(50):
        sbecodec.decode_batch(enc.out, enc.out_off, out=dec)
    h2 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"n={n}: pack alone {res['enc'][0]:.1f} us, decode alone {res['dec'][1]:.1f} us, "
          f"in pairs pack {res['pair'][0]:.1f} / decode {res['pair'][1]:.1f} us; host per call: "
          f"encode {(h1 - h0) / 50 * 1e6:.1f} us, decode {(h2 - h1) / 50 * 1e6:.1f} us", flush=True)
