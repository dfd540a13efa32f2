"""Diagnostic: determinism / accuracy of the training backward's pieces at 65536 rows."""
import torch
from normalizingflow_amd import fcnn_grad
dev = torch.device("cuda", 0)
torch.manual_seed(0)
for B in (16384, 65536):
    g = torch.randn(B, 736, device=dev)
    hb = torch.randn(B, 104, device=dev)
    h = hb[:, :101]
    ref = (g.double().t() @ h.double()).float()
    a = fcnn_grad.wgrad(g, h)
    b = fcnn_grad.wgrad(g, h)
    print(B, "wgrad rep maxdiff", (a - b).abs().max().item(), "vs fp64", (a - ref).abs().max().item(),
          "ref max", ref.abs().max().item())
    x = torch.randn(B, 64, device=dev)
    xs = x[:, 0::2][:, :32]
    ga1 = torch.randn(B, 100, device=dev)
    refx = (ga1.double().t() @ xs.double()).float()
    a = fcnn_grad.wgrad(ga1, xs)
    print(B, "wgrad strided maxdiff vs fp64", (a - refx).abs().max().item())
    W = torch.randn(736, 100, device=dev) * 0.1
    hh = torch.rand(B, 100, device=dev) * 2 - 1
    d1 = fcnn_grad.dh(g, W, hh)
    d2 = fcnn_grad.dh(g, W, hh)
    refd = ((g.double() @ W.double()) * (1 - hh.double() ** 2)).float()
    print(B, "dh rep maxdiff", (d1 - d2).abs().max().item(), "vs fp64", (d1 - refd).abs().max().item())
    s1 = g.sum(0); s2 = g.sum(0)
    print(B, "sum rep", (s1 - s2).abs().max().item())
