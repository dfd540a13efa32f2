"""Diagnostic: run-to-run determinism of one NSF_CL layer's backward pieces (c3 layer shape)."""
import torch
import nf.flows as nff
from normalizingflow_amd import kernels as K_
dev = torch.device("cuda", 0)
torch.manual_seed(3)
layer = nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[0]).to(dev)
import os
for B in [int(v) for v in os.environ.get('DBG_ROWS', '32768,65536,262144,1048576').split(',')]:
    x = torch.randn(B, 64, generator=torch.Generator().manual_seed(B)).to(dev) * 1.2
    gz = torch.randn(B, 64, device=dev) * 1e-3
    gld = torch.full((B,), -1.0 / B, device=dev)
    names = tuple(n for n, _ in layer.named_parameters())
    params = [p for _, p in layer.named_parameters()]
    need = (True,) + (True,) * len(params)
    outs = []
    for rep in range(3):
        r = layer._vjp(x, names, params, gz, gld, False, need)
        torch.cuda.synchronize()
        outs.append([t.clone() for t in r])
    for rep in (1, 2):
        d = [(a - b).abs().max().item() for a, b in zip(outs[0], outs[rep])]
        print(B, "rep", rep, "maxdiff gx %.3g" % d[0], " params", ["%.3g" % v for v in d[1:]])
    # the fused VJP kernel alone
    maps = layer._maps(dev)
    vpack = layer._vjp_pack(dev)
    H = layer.__dict__["_vjp_cache"][2]
    ldh = (H + 4) // 4 * 4
    res = []
    for rep in range(2):
        hbuf = torch.full((2, B, ldh), float("nan"), device=dev)
        gp = torch.full((B, 32 * 23), float("nan"), device=dev)
        gx = torch.full_like(x, float("nan"))
        K_.fused_nsf_vjp(x, vpack, maps.up_in, maps.up_out, maps.lo_in, maps.lo_out, H, gz, gld, gp, gx,
                         hbuf[0], hbuf[1], K=8, tail_bound=3.0, inverse=False)
        torch.cuda.synchronize()
        res.append((gp.clone(), gx.clone(), hbuf[0][:, :H + 1].clone(), hbuf[1][:, :H + 1].clone()))
    for i, nm in enumerate(("gp", "gx", "h1", "h2")):
        a, b = res[0][i], res[1][i]
        print(B, "kernel", nm, "nan", int(torch.isnan(a).sum()), "rep eq", torch.equal(a, b))
