"""Diagnostic: the fused NSF_AR at H = 354 (one wave per SIMD, 2-tile sub-records) vs
the oracle and the per-column path, run-to-run, per column."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nf.flows as nff  # noqa: E402
from normalizingflow_amd import config  # noqa: E402
from oracle import nf_oracle as orc  # noqa: E402

dev = torch.device("cuda", 0)
config.STRICT_CHECKS = False
from normalizingflow_amd import kernels as K_  # noqa: E402
for H, dim in [(int(h), int(d)) for h in os.environ.get("DBG_HS", "354").split(",")
               for d in os.environ.get("DBG_DIMS", "2,3,8,33,96").split(",")]:
    if not K_.fused_ar_supported(dim, H, 32):
        print("H %d dim %d: no fused instance" % (H, dim))
        continue
    torch.manual_seed(5)
    layer = nff.NSF_AR(dim=dim, K=32, B=1.462, hidden_dim=H)
    sd = {k: v.detach().cpu() for k, v in layer.state_dict().items()}
    layer = layer.to(dev)
    x = torch.randn(64, dim, generator=torch.Generator().manual_seed(1)) * 0.9
    z_ref, ld_ref = orc.nsf_ar(x, sd, "", dim, 32, 1.462)
    with torch.no_grad():
        z1, _ = layer(x.to(dev))
        z2, _ = layer(x.to(dev))
        prev = config.USE_FUSED
        config.USE_FUSED = False
        layer.invalidate_caches()
        zu, _ = layer(x.to(dev))
        config.USE_FUSED = prev
        layer.invalidate_caches()
    e = (z1.cpu() - z_ref).abs().amax(0)
    eu = (zu.cpu() - z_ref).abs().amax(0)
    print("H %d dim %d: fused rep-eq %s, fused err per column %s, max %.3g; unfused max %.3g" % (
        H, dim, torch.equal(z1, z2), ["%.2g" % v for v in e[:6].tolist()], float(e.max()), float(eu.max())), flush=True)
