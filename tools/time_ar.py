"""Time one fused NSF_AR layer launch (HIP events around the layer call) at the
applications' shapes: forward at the training batch, inverse at sample(500)
(applications/examples/fe.py:38-42).  usage: time_ar.py [dim H K rows_fwd rows_inv]"""
import sys

import torch

sys.path.insert(0, ".")
import nf.flows as nff  # noqa: E402

dev = torch.device("cuda", 0)
dim, H, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (96, 354, 32)))
rf, ri = (int(v) for v in (sys.argv[4:6] if len(sys.argv) > 5 else (40, 500)))
torch.manual_seed(0)
layer = nff.NSF_AR(dim=dim, K=K, B=1.5, hidden_dim=H).to(dev)


def timed(fn, n=30):
    with torch.no_grad():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


xf = torch.randn(rf, dim, device=dev) * 0.5
xi = torch.randn(ri, dim, device=dev) * 0.5
print("NSF_AR dim %d H %d K %d: forward %d rows %.4f ms per layer call, inverse %d rows %.4f ms" % (
    dim, H, K, rf, timed(lambda: layer(xf)), ri, timed(lambda: layer.inverse(xi))))
