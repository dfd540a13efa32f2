#!/usr/bin/env python
"""Static instruction mix of one kernel in a gfx950 assembly dump.

    hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off --cuda-device-only \
        -S normalizingflow_amd/csrc/nfk_fused_ksh25.hip -o /tmp/ksh25.s
    python tools/isa_mix.py /tmp/ksh25.s 'k_fused_nsfILi25ELi8ELb0' [--blocks]

Counts instructions per class for the whole kernel and per basic block
(labels), so the loop body of the chunk loop can be read off directly.
Also prints the kernel's resource metadata (.vgpr_count, .sgpr_count, spills)."""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")):
        return "trans"
    if op.startswith(("v_accvgpr",)):
        return "accmov"
    if op.startswith("v_cndmask"):
        return "cndmask"
    if op.startswith(("v_cmp", "v_cmpx")):
        return "vcmp"
    if re.match(r"v_\w+_f64", op) or op.startswith("v_cvt_f64") or op.startswith("v_cvt_f32_f64"):
        return "f64"
    if op.startswith("v_mov") or op.startswith("v_pk_mov"):
        return "vmov"
    if op.startswith("v_pk_"):
        return "vpk"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_barrier",)):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, pat = sys.argv[1], sys.argv[2]
    blocks = "--blocks" in sys.argv
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_Z\w*%s\w*:" % re.escape(pat), l):
            start = i
            name = l[:-1]
            break
    if start is None:
        sys.exit("kernel not found")
    end = start + 1
    while end < len(lines) and not lines[end].startswith(".Lfunc_end"):
        end += 1
    total = Counter()
    per = []
    cur_label, cur = "entry", Counter()
    for l in lines[start + 1:end]:
        s = l.strip()
        if not s or s.startswith((";", ".")) and not s.startswith(".LBB"):
            continue
        if s.startswith(".LBB") and s.endswith(":"):
            per.append((cur_label, cur))
            cur_label, cur = s[:-1], Counter()
            continue
        op = s.split()[0]
        c = classify(op)
        total[c] += 1
        cur[c] += 1
    per.append((cur_label, cur))
    print(name)
    print("  total:", dict(total.most_common()))
    meta = "\n".join(lines[end:end + 400])
    for key in ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                "group_segment_fixed_size", "private_segment_fixed_size"):
        m = re.search(r"\.%s:\s+(\d+)" % key, meta)
        if m:
            print("  %s: %s" % (key, m.group(1)))
    if blocks:
        for lab, c in per:
            n = sum(c.values())
            if n >= 40:
                print("  %-12s %5d  %s" % (lab, n, dict(c.most_common())))


if __name__ == "__main__":
    main()
