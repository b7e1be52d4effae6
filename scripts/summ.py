"""One-line summary of a bench JSON line on stdin (diagnosis helper)."""
import json
import sys

d = json.loads(sys.stdin.read().strip().splitlines()[-1])
k = d["kernels"]
print(f"{sys.argv[1] if len(sys.argv) > 1 else ''}: value={d['value']:.4g} ms/step={d['ms_per_step']:.4f} "
      f"pack={k['pack_ms']*1e3:.1f}us ({k['pack_gbs']:.0f} GB/s) dec={k['decode_kernel_ms']*1e3:.1f}us "
      f"({k['decode_kernel_gbs']:.0f} GB/s) enc_call={k['encode_ms']*1e3:.1f}us dec_call={k['decode_ms']*1e3:.1f}us "
      f"frac={d['roofline']['frac']:.3f}")
