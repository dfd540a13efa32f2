"""Diagnostic (tools only): in a gfx950 .s function body, list each packed-fp32
VALU instruction whose VGPR source was written by a transcendental
(v_exp/v_log/v_rcp/v_rsq/v_sqrt/v_sin/v_cos) within the previous N issued
instructions (straight-line distance, labels reset nothing), with the gap."""
import re
import sys
from collections import Counter

TRANS = re.compile(r"^v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32")


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return [int(m.group(1))] if m else []


def main(path, N=4):
    lines = [l.strip() for l in open(path)]
    hist = Counter()
    recent = []  # (index, op, dst regs)
    idx = 0
    for l in lines:
        if not l or l.startswith((";", ".")) or l.endswith(":"):
            continue
        parts = l.split(None, 1)
        op = parts[0]
        ops = [t.strip() for t in parts[1].split(",")] if len(parts) > 1 else []
        ops = [t.split()[0] if t else t for t in ops]
        if op.startswith("v_pk_") and op.endswith("f32"):
            srcs = set(r for t in ops[1:] for r in regs(t))
            for (j, wop, dst) in reversed(recent):
                if idx - j > N:
                    break
                if srcs & set(dst):
                    hist[(wop.split("_e")[0], op, idx - j)] += 1
                    break
        if op.startswith("v_") and ops:
            recent.append((idx, op, regs(ops[0])))
            recent = recent[-16:]
        idx += 1
    for k, v in sorted(hist.items(), key=lambda kv: kv[0][2]):
        if TRANS.match(k[0]):
            print("  %-14s -> %-14s gap %d : %d" % (k[0], k[1], k[2], v))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(p)
        main(p)
