"""Kernel variants by compile-time macro (no source edits): builds the product source
(aeron-cluster-client-cpp_amd/csrc/sbe_codec.hip) with extra -D flags into abl/<name>.so for
scripts/ab_rows.py.  Usage: python scripts/abv.py name=-DFOO=1,-DBAR=2 [name=...]  (base: no flags)"""
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "aeron-cluster-client-cpp_amd", "csrc", "sbe_codec.hip")
OUT = os.path.join(ROOT, "abl")


def build(spec):
    name, _, flags = spec.partition("=")
    os.makedirs(OUT, exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           *[f for f in flags.split(",") if f], SRC, "-o", os.path.join(OUT, f"{name}.so"), "-ldl"]
    subprocess.check_call(cmd)
    return name


if __name__ == "__main__":
    with cf.ThreadPoolExecutor(4) as ex:
        for n in ex.map(build, sys.argv[1:]):
            print("built", n)
