"""Diagnostic: chain form 2 (32x32x16) vs form 1 at growing batch sizes."""
import sys
import torch
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import nf.flows as nff
import nf.models as nfm
from normalizingflow_amd import _lib

lib = _lib.load()
dev = torch.device("cuda:0")
torch.manual_seed(1334)
flows = [nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[i % 2]) for i in range(8)]
model = nfm.NormalizingFlowModel(torch.distributions.MultivariateNormal(torch.zeros(64), torch.eye(64)), flows).to(dev)
model.prior = torch.distributions.MultivariateNormal(torch.zeros(64, device=dev), torch.eye(64, device=dev))
g = torch.Generator(device=dev).manual_seed(0)
xall = torch.randn(1 << 16, 64, device=dev, generator=g) * 1.2
for n in (128, 256, 4096, 8192, 32768, 65536):
    x = xall[:n].contiguous()
    res = {}
    for form in (1, 2):
        lib.nfk_debug_chain_form(form)
        with torch.no_grad():
            z, pl, ld = model(x)
            xi, ldi = model.inverse(x)
            xr, ldr = model.inverse(z)
        torch.cuda.synchronize()
        res[form] = (z, ld, xi, ldi, xr)
        assert lib.nfk_debug_last_chain_form() == form
    d = [float((a - b).abs().max()) for a, b in zip(res[1], res[2])]
    bad = (res[1][0] - res[2][0]).abs().amax(1) > 1e-3
    print(n, "z %.2e ld %.2e xi %.2e ldi %.2e xr %.2e" % tuple(d), "rt1 %.2e rt2 %.2e" % (
        float((res[1][4] - x).abs().max()), float((res[2][4] - x).abs().max())),
        "bad z rows", int(bad.sum()), bad.nonzero()[:8].flatten().tolist(), flush=True)
