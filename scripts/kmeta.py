"""Print per-kernel resource usage from a hipcc -S device assembly file (amdhsa metadata)."""
import re
import sys

txt = open(sys.argv[1]).read()
meta = txt[txt.index("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    name = g("name")
    if len(sys.argv) > 2 and not re.search(sys.argv[2], name):
        continue
    print(f"{name[:60]:60s} vgpr={g('vgpr_count')} sgpr={g('sgpr_count')} vspill={g('vgpr_spill_count')} "
          f"sspill={g('sgpr_spill_count')} lds={g('group_segment_fixed_size')} scratch={g('private_segment_fixed_size')}")
