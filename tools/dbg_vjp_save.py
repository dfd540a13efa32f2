"""Diagnostic (round 5): where does the fused VJP's run-to-run divergence enter?

Needs a library whose nfk_fused_vjp.hip was built with -DNFK_VJP_DIAG_SAVE
(tools/build_vjp_variant.sh NAME -DNFK_VJP_DIAG_SAVE [...]; NFK_LIBRARY selects
it): the kernel then also stores every element backward's INPUTS (the W, H, D
logits it recomputed on the matrix cores, x, dL/dz, dL/dlog|det|) next to its
outputs.  One clean launch, then DBG_REPS launches each after the register
file is poisoned with NaN (tools/libpoison.so).  Per rep:
  * inputs that differ from the clean launch's  -> the divergence is upstream
    of the element backward (recompute GEMMs, LDS, the x tile);
  * outputs that differ while the inputs are bitwise equal -> it is inside
    the element backward's own code.
For the differing elements the saved inputs are run through the unfused
backward kernel (nfk_rqs_coupling_bwd, exact element math) and through the
oracle's spline under fp64 autograd, and a few are printed.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nf.flows as nff  # noqa: E402
from normalizingflow_amd import _lib  # noqa: E402
from normalizingflow_amd import kernels as K_  # noqa: E402
from oracle import nf_oracle as orc  # noqa: E402

dev = torch.device("cuda", 0)
_P = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpoison.so"))
_P.poison_registers.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p]
KK, TB = 8, 3.0
P = 3 * KK - 1


def poison():
    rc = _P.poison_registers(16384, 0x7FC00000, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc


def elem_fp64(inp, inverse):
    """dL/dx and dL/dlogits of one NSF_CL spline element per row of inp
    ([N, 3K + 2]: logits, x, dL/dz, dL/dlog|det|) by fp64 autograd through the
    oracle (nf/flows.py:231-239 param handling, nf/utils.py:27-152)."""
    inp = inp.double()
    lg = inp[:, :P].clone().requires_grad_(True)
    x = inp[:, P].clone().requires_grad_(True)
    go, gl = inp[:, P + 1], inp[:, P + 2]
    W = 2 * TB * torch.softmax(lg[:, :KK], -1)
    H = 2 * TB * torch.softmax(lg[:, KK:2 * KK], -1)
    D = torch.nn.functional.softplus(lg[:, 2 * KK:])
    z, ld = orc.unconstrained_rq_spline(x, W, H, D, inverse=inverse, tail_bound=TB)
    (z * go + ld * gl).sum().backward()
    return x.grad, lg.grad


def main():
    lib = _lib.load()
    lib.nfk_vjp_diag_set.argtypes = [ctypes.c_void_p]
    lib.nfk_vjp_diag_set.restype = ctypes.c_int
    torch.manual_seed(3)
    layer = nff.NSF_CL(size=32, dim=2, K=KK, B=TB, hidden_dim=100, mask=[0]).to(dev)
    maps = layer._maps(dev)
    vpack = layer._vjp_pack(dev)
    H = layer.__dict__["_vjp_cache"][2]
    ldh = (H + 4) // 4 * 4
    reps = int(os.environ.get("DBG_REPS", "3"))
    for inverse in [bool(int(v)) for v in os.environ.get("DBG_INV", "1,0").split(",")]:
        for B in [int(v) for v in os.environ.get("DBG_ROWS", "262144").split(",")]:
            x = torch.randn(B, 64, generator=torch.Generator().manual_seed(B)).to(dev) * 1.2
            gz = torch.randn(B, 64, generator=torch.Generator().manual_seed(B + 1)).to(dev) * 1e-3
            gld = torch.full((B,), -1.0 / B, device=dev)
            hbuf = torch.zeros(2, B, ldh, device=dev)
            gp = torch.zeros(B, 32 * P, device=dev)
            gx = torch.zeros_like(x)
            dbg = torch.zeros(B * 32, 3 * KK + 2, device=dev)
            assert lib.nfk_vjp_diag_set(ctypes.c_void_p(dbg.data_ptr())) == 0

            def run(do_poison):
                for t in (hbuf, gp, gx, dbg):
                    t.zero_()
                torch.cuda.synchronize()
                if do_poison:
                    poison()
                K_.fused_nsf_vjp(x, vpack, maps.up_in, maps.up_out, maps.lo_in, maps.lo_out, H, gz, gld, gp, gx,
                                 hbuf[0], hbuf[1], K=KK, tail_bound=TB, inverse=inverse)
                torch.cuda.synchronize()
                return gp.view(B * 32, P).clone(), gx.clone(), dbg.clone()

            c_gp, c_gx, c_in = run(False)
            print("inv=%d B=%d clean: gp nan %d, inputs nan %d" % (inverse, B, int(torch.isnan(c_gp).sum()),
                                                                    int(torch.isnan(c_in).sum())), flush=True)
            counts = getattr(lib, "nfk_vjp_diag_counts", None)
            if counts is not None:
                counts.argtypes = [ctypes.c_void_p, ctypes.c_int]
                cbuf = (ctypes.c_int * (64 + 80))()
                counts(ctypes.cast(cbuf, ctypes.c_void_p), 1)
            for rep in range(reps):
                r_gp, r_gx, r_in = run(True)
                if counts is not None:
                    counts(ctypes.cast(cbuf, ctypes.c_void_p), 1)
                    print("  twice: per-lane mismatches of the two evaluations: total %d, lanes 0-47 %d, "
                          "48-63 %d" % (sum(cbuf[:64]), sum(cbuf[:48]), sum(cbuf[48:64])), flush=True)
                    firsts = {i: cbuf[64 + i] for i in range(80) if cbuf[64 + i]}
                    if firsts:
                        print("  probe: first differing intermediate slot -> count %s" % firsts, flush=True)
                in_diff = (r_in != c_in) & ~(torch.isnan(r_in) & torch.isnan(c_in))
                out_diff = (r_gp != c_gp) & ~(torch.isnan(r_gp) & torch.isnan(c_gp))
                el_in = in_diff.any(1)
                el_out = out_diff.any(1)
                print("inv=%d B=%d rep %d: elements with differing inputs %d, differing outputs %d "
                      "(of which with equal inputs %d); gp nan %d; gx diff %.3g" % (
                          inverse, B, rep, int(el_in.sum()), int(el_out.sum()), int((el_out & ~el_in).sum()),
                          int(torch.isnan(r_gp).sum()), float((r_gx - c_gx).abs().nan_to_num(0).max())),
                      flush=True)
                for name, sel in (("diff-in", el_in), ("diff-out/eq-in", el_out & ~el_in)):
                    idx = sel.nonzero().flatten()
                    if idx.numel() == 0:
                        continue
                    rows = idx // 32
                    cols = idx % 32
                    print("  %s: rows mod 16 %s, row blocks (64) %s, coords %s, waves-in-WG %s" % (
                        name, sorted(set((rows % 16).tolist()))[:16], sorted(set((rows // 64).tolist()))[:10],
                        sorted(set(cols.tolist()))[:32], sorted(set(((rows // 16) % 4).tolist()))), flush=True)
                    which = in_diff[idx].float().sum(0) if name == "diff-in" else out_diff[idx].float().sum(0)
                    print("  %s: per-slot counts %s" % (name, which.long().tolist()), flush=True)
                    k = idx[:4]
                    for e in k.tolist():
                        print("    elem %d (row %d coord %d)\n      clean in  %s\n      rep   in  %s\n"
                              "      clean out %s\n      rep   out %s" % (
                                  e, e // 32, e % 32, c_in[e].tolist(), r_in[e].tolist(), c_gp[e].tolist(),
                                  r_gp[e].tolist()), flush=True)
                    # the saved inputs through the unfused exact kernel and fp64 autograd
                    sel_in = r_in[idx[:4096]]
                    n = sel_in.shape[0]
                    xs = sel_in[:, P:P + 1].contiguous()
                    prm = sel_in[:, :P].contiguous().view(n, 1, P)
                    gzs = sel_in[:, P + 1:P + 2].contiguous()
                    gls = sel_in[:, P + 2].contiguous()
                    gprm = torch.zeros_like(prm)
                    gxs = torch.zeros_like(xs)
                    col = torch.zeros(1, dtype=torch.int32, device=dev)
                    K_.rqs_coupling_bwd(xs, prm, col, col, gzs, gls, gprm, gxs, K=KK, left=-TB, right=TB,
                                        bottom=-TB, top=TB, tails=True, param_mode=0, inverse=inverse)
                    torch.cuda.synchronize()
                    gx64, gp64 = elem_fp64(sel_in.cpu(), inverse)
                    rg = r_gp[idx[:4096]].cpu().double()
                    print("  %s: unfused kernel on the rep's inputs vs rep outputs: max |d| %.3g; "
                          "vs fp64: unfused %.3g, rep %.3g, clean %.3g" % (
                              name, float((gprm.view(n, P).cpu().double() - rg).abs().nan_to_num(1e30).max()),
                              float((gprm.view(n, P).cpu().double() - gp64).abs().nan_to_num(1e30).max()),
                              float((rg - gp64).abs().nan_to_num(1e30).max()),
                              float((c_gp[idx[:4096]].cpu().double() - gp64).abs().nan_to_num(1e30).max())),
                          flush=True)


if __name__ == "__main__":
    main()
