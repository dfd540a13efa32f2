"""Insert s_nop 0 between a packed-FP32 (or 64-bit VALU) write and a packed-FP32 read of it at gap 1 in an AMDGPU .s file."""
import re, sys
def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m: return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()
src, dst = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
out, prev, n = [], None, 0
for l in lines:
    s = l.split(";")[0].strip()
    parts = s.split(None, 1)
    op = parts[0] if parts else ""
    ops = [t.strip().split()[0] for t in parts[1].split(",")] if len(parts) > 1 and parts[1].strip() else []
    is_ins = bool(op) and not op.startswith(".") and not op.endswith(":")
    if is_ins and op.startswith("v_pk_") and op.endswith("f32") and prev is not None:
        if any(prev & regs(t) for t in ops[1:]):
            out.append("\ts_nop 0")
            n += 1
    out.append(l)
    if is_ins:
        if op.startswith("v_") and ops and (op.startswith("v_pk_") or "_b64" in op or "_f64" in op):
            prev = regs(ops[0])
        else:
            prev = None
    elif s.endswith(":"):
        prev = None
open(dst, "w").write("\n".join(out))
print("inserted", n)
