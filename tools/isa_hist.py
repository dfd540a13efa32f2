"""Instruction histogram of one kernel in a hipcc --cuda-device-only -S listing.

usage: python tools/isa_hist.py listing.s kernel-substring [kernel-substring ...]
Counts MFMAs, AGPR copies, LDS reads/writes, scratch accesses, VALU and s_waitcnt.
"""
import re
import sys

src = open(sys.argv[1]).read()
for key in sys.argv[2:]:
    m = re.search(r"^(\S*%s\S*):.*?\n(.*?)\.Lfunc_end" % re.escape(key), src, re.S | re.M)
    if not m:
        print(key, "not found")
        continue
    body = m.group(2)

    def cnt(p):
        return len(re.findall(p, body, re.M))

    print(m.group(1)[:80])
    print("  mfma %d (agpr dst %d)  accvgpr_read %d  accvgpr_write %d  ds_read %d  ds_write %d  scratch %d"
          "  valu %d  salu %d  s_waitcnt %d  s_barrier %d" % (
              cnt(r"^\s+v_mfma"), cnt(r"^\s+v_mfma\S*\s+a\["), cnt(r"^\s+v_accvgpr_read"),
              cnt(r"^\s+v_accvgpr_write"), cnt(r"^\s+ds_read"), cnt(r"^\s+ds_write"), cnt(r"^\s+scratch_"),
              cnt(r"^\s+v_"), cnt(r"^\s+s_"), cnt(r"^\s+s_waitcnt"), cnt(r"^\s+s_barrier")))
