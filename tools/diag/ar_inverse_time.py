"""Diagnostic: time the fused NSF_AR inverse (sample direction) at 2^20 rows."""
import sys
import torch
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import nf.flows as nff
from normalizingflow_amd import flush_status_checks

dev = torch.device("cuda:0")
torch.manual_seed(1234)
layer = nff.NSF_AR(dim=40, K=10, B=4.0, hidden_dim=80).to(dev)
x = torch.randn(1 << 20, 40, device=dev)
with torch.no_grad():
    for _ in range(2):
        layer.inverse(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        layer.inverse(x)
    e1.record()
    torch.cuda.synchronize()
flush_status_checks()
print("ar inverse ms per layer: %.3f" % (e0.elapsed_time(e1) / 5))
