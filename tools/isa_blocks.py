"""Per-basic-block MFMA / VALU / LDS counts of one kernel in a hipcc -S listing,
and how often the instruction stream switches between MFMA and VALU (a
measure of interleaving).  usage: python tools/isa_blocks.py listing.s kernel-substring [min_mfma]"""
import re
import sys

src = open(sys.argv[1]).read()
m = re.search(r"^(\S*%s\S*):.*?\n(.*?)\.Lfunc_end" % re.escape(sys.argv[2]), src, re.S | re.M)
min_m = int(sys.argv[3]) if len(sys.argv) > 3 else 1
cur, name = [], "entry"
blocks = []
for l in m.group(2).split("\n"):
    if l.startswith(".LBB"):
        blocks.append((name, cur))
        cur, name = [], l.split(":")[0]
        continue
    cur.append(l)
    if re.match(r"\s+s_(cbranch|branch|barrier)", l):
        blocks.append((name, cur))
        cur, name = [], name + "+"
blocks.append((name, cur))
for n, b in blocks:
    v = [l for l in b if re.match(r"\s+v_", l) and not re.match(r"\s+v_accvgpr", l)]
    mf = sum(1 for l in v if "v_mfma" in l)
    if mf < min_m:
        continue
    seq = ["M" if "v_mfma" in l else "V" for l in v]
    sw = sum(1 for i in range(1, len(seq)) if seq[i] != seq[i - 1])
    print("%-12s mfma %4d valu %4d trans %3d ds %3d scratch %2d switches %3d" % (
        n, mf, len(v) - mf, sum(1 for l in v if re.match(r"\s+v_(exp|log|rcp|sqrt|rsq)", l)),
        sum(1 for l in b if re.match(r"\s+ds_", l)), sum(1 for l in b if re.match(r"\s+scratch", l)), sw))
