"""Diagnostic: run-to-run determinism of one NSF_CL layer's backward with the
fused VJP kernel on and off (config.USE_FUSED_VJP), c3 layer shape."""
import torch
import nf.flows as nff
from normalizingflow_amd import config
dev = torch.device("cuda", 0)
torch.manual_seed(3)
layer = nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[0]).to(dev)
names = tuple(n for n, _ in layer.named_parameters())
params = [p for _, p in layer.named_parameters()]
for B in (4097, 262144):
    x = torch.randn(B, 64, generator=torch.Generator().manual_seed(B)).to(dev) * 1.2
    gz = torch.randn(B, 64, device=dev) * 1e-3
    gld = torch.full((B,), -1.0 / B, device=dev)
    for fused in (True, False):
        config.USE_FUSED_VJP = fused
        outs = [[t.clone() for t in layer._vjp(x, names, params, gz, gld, False, (True,) * 7)] for _ in range(3)]
        d = max(max((a - b).abs().max().item() for a, b in zip(outs[0], outs[r])) for r in (1, 2))
        print("rows %d fused_vjp %s: max run-to-run difference over 3 runs %.3g" % (B, fused, d))
