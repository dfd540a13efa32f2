"""Resource metadata (VGPR/AGPR/SGPR/spills/LDS) of kernels in a gfx950 asm dump.

    python tools/kres.py dump.s [name-substring]
"""
import re
import sys

text = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
meta = text[text.find("amdhsa.kernels:"):]
for blk in meta.split("\n  - ")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or pat not in name.group(1):
        continue
    f = {k: re.search(r"\." + k + r":\s+(\d+)", blk) for k in
         ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
          "group_segment_fixed_size", "private_segment_fixed_size")}
    print(name.group(1), " ".join("%s=%s" % (k, v.group(1)) for k, v in f.items() if v))
