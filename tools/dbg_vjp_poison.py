"""Diagnostic: does a kernel read a register it never wrote?

Every VGPR/AGPR of every SIMD is filled with a quiet NaN (tools/libpoison.so)
right before the launch; an uninitialised register read then turns into NaN
outputs (deterministically, at any batch size) instead of a value some earlier
wave left behind (run-to-run different, only when waves share a SIMD).
Part 1: nfk_fused_nsf_vjp at the c3 layer shape, both directions.
Part 2: every bench workload's log_prob (and c3's sample), poisoned vs clean.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nf.flows as nff  # noqa: E402
from normalizingflow_amd import kernels as K_  # noqa: E402

dev = torch.device("cuda", 0)
_P = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpoison.so"))
_P.poison_registers.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p]


def poison():
    rc = _P.poison_registers(16384, 0x7FC00000, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc


def vjp_part(rows_list, reps):
    torch.manual_seed(3)
    layer = nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[0]).to(dev)
    maps = layer._maps(dev)
    vpack = layer._vjp_pack(dev)
    H = layer.__dict__["_vjp_cache"][2]
    ldh = (H + 4) // 4 * 4
    for inverse in (False, True):
        for B in rows_list:
            x = torch.randn(B, 64, generator=torch.Generator().manual_seed(B)).to(dev) * 1.2
            gz = torch.randn(B, 64, generator=torch.Generator().manual_seed(B + 1)).to(dev) * 1e-3
            gld = torch.full((B,), -1.0 / B, device=dev)
            hbuf = torch.zeros(2, B, ldh, device=dev)
            gp = torch.zeros(B, 32 * 23, device=dev)
            gx = torch.zeros_like(x)

            def run(do_poison):
                hbuf.zero_()
                gp.zero_()
                gx.zero_()
                torch.cuda.synchronize()
                if do_poison:
                    poison()
                K_.fused_nsf_vjp(x, vpack, maps.up_in, maps.up_out, maps.lo_in, maps.lo_out, H, gz, gld, gp, gx,
                                 hbuf[0], hbuf[1], K=8, tail_bound=3.0, inverse=inverse)
                torch.cuda.synchronize()
                return [gp.clone(), gx.clone(), hbuf[0][:, :H + 1].clone(), hbuf[1][:, :H + 1].clone()]

            ref = run(False)
            for rep in range(reps):
                out = run(True)
                msg = []
                for nm, a, r in zip(("gp", "gx", "h1", "h2"), out, ref):
                    nan = torch.isnan(a)
                    d = (a - r).abs()
                    d[nan] = 0
                    msg.append("%s nan %d diff %.3g" % (nm, int(nan.sum()), float(d.max())))
                    if nan.any() and rep == 0:
                        rr, cc = nan.nonzero(as_tuple=True)
                        print("   %s NaN rows mod 16 %s, row blocks %s, cols %s" % (
                            nm, sorted(set((rr % 16).tolist()))[:16], sorted(set((rr // 64).tolist()))[:8],
                            sorted(set(cc.tolist()))[:40] if nm != "gp" else
                            sorted(set((cc % 23).tolist()))), flush=True)
                print("vjp inv=%d B=%d rep %d: %s" % (inverse, B, rep, "; ".join(msg)), flush=True)


def model_part(n):
    import bench
    for wl in ("c3", "c2", "c5", "c1", "ar"):
        try:
            torch.manual_seed(0)
            model = bench.build_model(wl, dev)[0]
            rows = 4096 if wl == "c1" else n
            x = bench.make_x(wl, rows, torch.Generator().manual_seed(1), "cpu").to(dev)
            with torch.no_grad():
                ref = model.log_prob(x).clone()
                torch.cuda.synchronize()
                for rep in range(2):
                    poison()
                    lp = model.log_prob(x)
                    torch.cuda.synchronize()
                    print("model %s rows %d rep %d: log_prob nan %d (clean nan %d), diff %.3g" % (
                        wl, rows, rep, int(torch.isnan(lp).sum()), int(torch.isnan(ref).sum()),
                        float((lp - ref).abs().nan_to_num(0).max())), flush=True)
                if wl == "c3":
                    z = torch.randn(rows, 64, generator=torch.Generator().manual_seed(2)).to(dev)
                    ref = model.inverse(z) if hasattr(model, "inverse") else None
                    ref = ref[0] if isinstance(ref, tuple) else ref
                    torch.cuda.synchronize()
                    poison()
                    o = model.inverse(z)
                    o = o[0] if isinstance(o, tuple) else o
                    torch.cuda.synchronize()
                    print("model c3 inverse nan %d diff %.3g" % (int(torch.isnan(o).sum()),
                                                                 float((o - ref).abs().nan_to_num(0).max())), flush=True)
        except Exception as e:  # report and go on to the next workload
            print("model %s: %s: %s" % (wl, type(e).__name__, e), flush=True)


if __name__ == "__main__":
    rows = [int(v) for v in os.environ.get("DBG_ROWS", "4097,65536,262144").split(",")]
    vjp_part(rows, int(os.environ.get("DBG_REPS", "2")))
    if os.environ.get("DBG_MODELS", "1") == "1":
        model_part(int(os.environ.get("DBG_MODEL_ROWS", "262144")))
