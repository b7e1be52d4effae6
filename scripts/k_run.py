"""Run the encode (pack) or the parse_message decode of one workload K times with a given library
build, for rocprofv3 PMC passes on one kernel.  Usage: python scripts/k_run.py LIB [--var] [--k K]
[--enc]  (default: decode; --enc: encode, K times)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "aeron-cluster-client-cpp_amd"), os.path.join(ROOT, "tests")]
import sbe_testlib as T  # noqa: E402
import sbecodec  # noqa: E402

sbecodec.use_library(os.path.abspath(sys.argv[1]))
sbecodec.require_device()
dev = torch.device("cuda:0")
var = "--var" in sys.argv
k = int(sys.argv[sys.argv.index("--k") + 1]) if "--k" in sys.argv else 5
n = 4194304 if var else 1_000_000
if var:
    a, l, t = T.var_orders_t(n, dev)
else:
    arena, L, ts = T.fixed256_orders(n)
    a, l, t = (torch.from_numpy(arena).to(dev), torch.from_numpy(L.view(np.int32)).to(dev),
               torch.from_numpy(ts.view(np.int64)).to(dev))
enc = sbecodec.encode_topic_batch(a, l, t)
if "--enc" in sys.argv:
    ws = sbecodec.alloc_workspace(n, dev)
    for _ in range(k):
        sbecodec.encode_topic_batch(a, l, t, out=enc.out, out_off=enc.out_off, status=enc.status, workspace=ws)
else:
    dec = sbecodec.alloc_decoded(n, dev)
    for _ in range(k):
        sbecodec.decode_batch(enc.out, enc.out_off, out=dec)
torch.cuda.synchronize()
print("ok", n, k)
