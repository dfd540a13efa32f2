"""Debug: per-column difference between the split and whole-record forms of the
fused NSF_CL layer kernel (a localising aid: which coordinates / registers differ)."""
import os, sys
import torch
sys.path.insert(0, ".")
import nf.flows as nff
from normalizingflow_amd import _lib

lib = _lib.load()
print("lib", _lib.LIB_PATH)
dev = torch.device("cuda:0")
for size, dim, K, H, mask in [(12, 2, 6, 33, [1]), (12, 2, 5, 33, [1]), (12, 2, 10, 100, [1]), (12, 2, 4, 130, [1]), (16, 2, 8, 33, [0])]:
    torch.manual_seed(size + 7 * K + H)
    layer = nff.NSF_CL(size=size, dim=dim, K=K, B=3, hidden_dim=H, mask=mask).to(dev)
    x = (torch.randn(64, size * dim, generator=torch.Generator().manual_seed(3)) * 1.3).to(dev)
    res = {}
    for f in (0, 1):
        lib.nfk_debug_fused_form(f)
        with torch.no_grad():
            res[f] = layer(x)[0].cpu()
    d = (res[0] - res[1]).abs()
    print("s%d K%d H%d: maxdiff %.3g; per column max:" % (size, K, H, float(d.max())))
    print(" ".join("%.1e" % v for v in d.max(0).values.tolist()))
    print("rows with diff:", int((d.max(1).values > 1e-4).sum()), "of", d.shape[0])
