"""Debug: nfk_fused_nsf_vjp's outputs (gp, gx, h1, h2) against the unfused
recompute (fcnn_grad.forward_saved + nfk_rqs_coupling_bwd) on one layer."""
import sys
import torch
sys.path.insert(0, ".")
import nf.flows as nff
from normalizingflow_amd import kernels as K_, fcnn_grad

dev = torch.device("cuda:0")
torch.manual_seed(3)
size, K, H, mask = 32, 8, 100, [0]
layer = nff.NSF_CL(size=size, dim=2, K=K, B=3, hidden_dim=H, mask=mask).to(dev)
B = 1037
x = torch.randn(B, 64, device=dev) * 1.2
gz = torch.randn(B, 64, device=dev)
gld = torch.randn(B, device=dev)
maps = layer._maps(dev)
vpack = layer._vjp_pack(dev)
ldh = (H + 4) // 4 * 4
hbuf = torch.full((2, B, ldh), float("nan"), device=dev)
gp = torch.full((B, 32 * (3 * K - 1)), float("nan"), device=dev)
gx = torch.full((B, 64), float("nan"), device=dev)
K_.fused_nsf_vjp(x, vpack, maps.up_in, maps.up_out, maps.lo_in, maps.lo_out, H, gz, gld, gp, gx, hbuf[0], hbuf[1],
                 K=K, tail_bound=3.0)
torch.cuda.synchronize()
p = {n: t.detach() for n, t in layer.named_parameters()}
lower = x.index_select(1, maps.lo_in_long)
raw, cache = fcnn_grad.forward_saved(p, "psi.", lower)
gp2 = torch.empty_like(gp)
gx2 = torch.empty_like(gx)
K_.rqs_coupling_bwd(x, raw.contiguous(), maps.up_in, maps.up_out, gz, gld, gp2, gx2, lo_in=maps.lo_in,
                    lo_out=maps.lo_out, K=K, left=-3.0, right=3.0, bottom=-3.0, top=3.0, tails=True, param_mode=0,
                    inverse=False)
torch.cuda.synchronize()
for name, a, b in (("h1", hbuf[0][:, :H + 1], cache[1]), ("h2", hbuf[1][:, :H + 1], cache[2]), ("gp", gp, gp2),
                   ("gx", gx, gx2)):
    d = (a - b).abs()
    print(name, "nan", int(torch.isnan(a).sum()), "max", float(d.nan_to_num(1e30).max()),
          "scale", float(b.abs().max()))
    if name in ("h1", "h2"):
        bad = (d.nan_to_num(1e30) > 1e-4).nonzero()
        print("  bad cols", sorted(set(bad[:, 1].tolist()))[:40], "rows", len(set(bad[:, 0].tolist())))
    if name == "gp":
        dd = d.nan_to_num(1e30).view(B, 32, 3 * K - 1).amax(dim=(0,))
        print("  per coord max", [round(float(v), 4) for v in dd.amax(1)])
        print("  per param max", [round(float(v), 4) for v in dd.amax(0)])
