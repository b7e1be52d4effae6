"""GPU probe: encode/decode at growing sizes with progress output (diagnosis helper)."""
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
ws = sbecodec.alloc_workspace(1 << 20, dev)
for gen, sizes in (("var", [1, 65, 640, 6400, 20000, 200000]), ("fixed", [100, 200000])):
    for n in sizes:
        arena, L, ts = (T.var_orders if gen == "var" else T.fixed256_orders)(n)
        for rep in range(3):
            t0 = time.time()
            enc = sbecodec.encode_topic_batch(torch.from_numpy(arena).to(dev), torch.from_numpy(L.view(np.int32)).to(dev),
                                              torch.from_numpy(ts.view(np.int64)).to(dev), workspace=ws)
            torch.cuda.synchronize()
            err = 0
            eo, eoff, _ = T.oracle_encode(arena, L, ts)
            off = enc.out_off.cpu().numpy().view(np.uint64)
            ok_off = np.array_equal(off, eoff)
            ok = ok_off and np.array_equal(enc.out[: int(off[-1])].cpu().numpy(), eo)
            print(f"{gen} n={n} rep={rep} err={err} offsets_ok={ok_off} bytes_ok={ok} {time.time()-t0:.2f}s", flush=True)
            if not ok_off:
                bad = np.nonzero(off != eoff)[0]
                print("  first bad offsets", bad[:5], off[bad[:5]], eoff[bad[:5]], flush=True)
