"""Timeline of the fused NSF kernels from a -DNFK_TRACE build.

NFK_LIBRARY=.../libnfk_trace.so python tools/trace_wide.py [--batch N] [--inverse]
    c5 layer (wide kernel, nfk_fused_wide.h)
NFK_LIBRARY=.../libnfk_trace.so python tools/trace_wide.py --c3
    c3 layer (narrow kernel, nfk_fused_impl.h): per phase "gemm" (previous mark
    -> GEMM issued), "epi" (-> epilogue done), "barrier" (-> barrier passed)

Every 512th workgroup records s_memtime at each mark of every wave
(nfk_fused_wide.h NFK_MARK): start, prologue done, per sub-step "GEMM
issued" and "barrier passed", per chunk the end of epilogues A, B, C, end.
Prints mean cycles per category: GEMM (previous mark -> GEMM issued),
barrier wait (GEMM issued -> barrier passed), epilogues, prologue.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nf.flows as nff  # noqa: E402
from normalizingflow_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--inverse", action="store_true")
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--K", type=int, default=16)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--c3", action="store_true")
    ap.add_argument("--slots1", action="store_true", help="c3 kernel built with NFK_NSF_SLOTS=1")
    ap.add_argument("--split", type=int, default=0,
                    help="c3 kernel in the split form with this many tiles per sub-record (NFK_SPLIT_NS)")
    ap.add_argument("--pipe", action="store_true", help="with --split: the pipelined schedule")
    args = ap.parse_args()
    if args.c3:
        args.size, args.K, args.hidden = 32, 8, 100
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    layer = nff.NSF_CL(size=args.size, dim=2, K=args.K, B=3, hidden_dim=args.hidden, mask=[0]).to(dev)
    x = torch.randn(args.batch, 2 * args.size, device=dev)
    nwg = (args.batch + 63) // 64  # workgroups of 4 or 8 waves: sized for 4
    slots = (nwg + 511) // 512
    buf = torch.zeros(slots * 16 * 260, dtype=torch.int32, device=dev)
    lib = _lib.load()
    lib.nfk_debug_trace.argtypes = [ctypes.c_void_p]
    lib.nfk_debug_trace(buf.data_ptr())
    with torch.no_grad():
        for _ in range(3):
            (layer.inverse(x) if args.inverse else layer(x))
    torch.cuda.synchronize()
    lib.nfk_debug_trace(None)
    t = buf.view(slots, 16, 260).cpu().numpy().astype(np.int64)
    waves = [(w, t[w // 16, w % 16]) for w in range(slots * 16) if t[w // 16, w % 16, 256] > 0]
    n = int(waves[0][1][256])
    marks = np.stack([v[:n] for _, v in waves])  # [waves, marks] 32-bit cycle counts
    d = np.diff(marks, axis=1) % (1 << 32)       # intervals
    tot = (marks[:, -1] - marks[:, 0]) % (1 << 32)
    # classify the intervals: 0 prologue-to-start... follow the mark order of the kernel
    S1, S2, SC = 2, 4, 2  # c5 shape (H=256, K=16, n_lo=128)
    cats = []
    ap_pipe = args.pipe
    if args.c3 and args.split and ap_pipe:
        # pipelined split schedule (NFK_SPLIT_PIPE): every GEMM part is followed
        # by half an epilogue; layer 2 as the plain split form
        cats.append("prologue")
        cats += ["gemm_L1", "bar_gemm", "epi_L1", "bar_epi"]
        cats += ["gemm_L2", "bar_gemm", "gemm_L2", "bar_gemm", "epi_L2", "bar_epi"]
        for ch in range((args.size + 15) // 16):
            for g, e in [("A", "C01prev" if ch else "none"), ("A", "A01"), ("B", "A23"), ("B", "B01"),
                         ("C", "B23"), ("C", "C01")]:
                cats += ["gemm_" + g, "bar_gemm", "epi_" + e[0] if e != "none" else "wait", "bar_epi"]
        cats.append("epiC23+tail")
    elif args.c3 and args.split:
        # per GEMM part: "gemm" (previous mark -> GEMM issued; includes the wait
        # for the part's copy), "bar_gemm"; per record: "epi", "bar_epi"
        ns = args.split
        parts = {"L1": 1, "L2": -(-7 // ns), "A": -(-8 // ns), "B": -(-8 // ns), "C": -(-7 // ns)}
        cats.append("prologue")
        for ph in ["L1", "L2"] + list("ABC") * ((args.size + 15) // 16):
            cats += ["gemm_" + ph, "bar_gemm"] * parts[ph] + ["epi_" + ph, "bar_epi"]
        cats.append("tail")
    elif args.c3:
        cats.append("prologue")
        for ph in ["L1", "L2"] + list("ABC") * ((args.size + 15) // 16):
            cats += (["gemm_" + ph, "bar_gemm", "epi_" + ph, "bar_epi"] if args.slots1
                     else ["gemm_" + ph, "epi_" + ph, "barrier"])
        cats.append("tail")
    elif args.hidden != 256 or args.K != 16 or args.size != 128:
        print("note: categories assume the c5 shape")
    for _ in range(0 if args.c3 else 1):
        cats.append("prologue")                       # start -> prologue done
    for _ in range(0 if args.c3 else S1 + S2):
        cats += ["gemm_L12", "barrier"]
    nch = 0 if args.c3 else (args.size + 7) // 8
    for _ in range(nch):
        for ph in "ABC":
            for _ in range(SC):
                cats += ["gemm_" + ph, "barrier"]
            cats.append("epi_" + ph)
    if not args.c3:
        cats.append("tail")
    cats = cats[:d.shape[1]]
    print("waves traced: %d, marks per wave: %d, mean wave cycles: %.0f" % (len(waves), n, tot.mean()))
    agg = {}
    for i, c in enumerate(cats):
        agg.setdefault(c, []).append(d[:, i])
    rows = []
    for c, v in agg.items():
        v = np.stack(v, axis=1)
        rows.append((c, v.shape[1], v.mean(), v.sum(axis=1).mean()))
    print("%-10s %6s %12s %14s %7s" % ("category", "count", "mean/cyc", "total/wave", "share"))
    for c, cnt, m, s in rows:
        print("%-10s %6d %12.0f %14.0f %6.1f%%" % (c, cnt, m, s, 100.0 * s / tot.mean()))
    # first chunk's per-interval detail for wave 0 of the first traced workgroup
    lo, hi = (0, d.shape[1]) if args.c3 else (13, min(28, d.shape[1]))
    print("intervals (wave mean):", " ".join("%s=%.0f" % (cats[i], d[:, i].mean()) for i in range(lo, hi)))


if __name__ == "__main__":
    main()
