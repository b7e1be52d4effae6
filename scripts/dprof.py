"""Phase profile of the decode kernel from an instrumented build (abl/dprof.so: per-wave
s_memtime deltas summed per phase).  Usage: python scripts/dprof.py abl/dprof.so [--var]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "aeron-cluster-client-cpp_amd"), os.path.join(ROOT, "tests")]
import sbe_testlib as T  # noqa: E402
import sbecodec  # noqa: E402

lib_path = os.path.abspath(sys.argv[1])
sbecodec.use_library(lib_path)
sbecodec.require_device()
lib = ctypes.CDLL(lib_path)
dev = torch.device("cuda:0")
var = "--var" in sys.argv
n = 4194304 if var else 1_000_000
if var:
    a, l, t = T.var_orders_t(n, dev)
else:
    arena, L, ts = T.fixed256_orders(n)
    a, l, t = (torch.from_numpy(arena).to(dev), torch.from_numpy(L.view(np.int32)).to(dev),
               torch.from_numpy(ts.view(np.int64)).to(dev))
enc = sbecodec.encode_topic_batch(a, l, t)
dec = sbecodec.alloc_decoded(n, dev)
for _ in range(3):
    sbecodec.decode_batch(enc.out, enc.out_off, out=dec)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 24)()
lib.sbe_dprof_read(buf)
K = 5
for _ in range(K):
    sbecodec.decode_batch(enc.out, enc.out_off, out=dec)
torch.cuda.synchronize()
lib.sbe_dprof_read(buf)
v = np.array(buf[:8], dtype=np.float64)  # parse_message mode
if "--count" in sys.argv:
    names = ["windows", "lane_path", "win_scan", "more_fallback", "hit_iters", "-", "scan_bytes", "waves"]
    w = v[7]
    print(f"{'var' if var else 'fixed'} per wave: " + " ".join(f"{names[k]}={v[k] / w:.3f}" for k in range(7)))
    sys.exit(0)
waves = v[7]
names = ["stage1", "parse", "seq", "stageN", "stores", "windowsN", "total", "waves"]
print(f"{'var' if var else 'fixed'}: waves {waves:.0f}, later windows per wave {v[5] / waves:.2f}")
for k in (0, 1, 2, 3, 4, 6):
    print(f"  {names[k]:8s} {v[k] / waves:10.0f} cycles/wave  {v[k] / v[6] * 100:5.1f} %")
