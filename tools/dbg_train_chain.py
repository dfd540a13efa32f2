"""Diagnostic: determinism of x.grad in the c3-like train step, chain vs per-layer (2 layers)."""
import sys
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_gpu_train_chain as t


class MP:
    def setattr(self, obj, name, val):
        setattr(obj, name, val)


dev = torch.device("cuda", 0)
for rows in (4097, 65536):
    model = t._model(2, dev)
    x = torch.randn(rows, 64, generator=torch.Generator().manual_seed(rows)).to(dev) * 1.2
    import normalizingflow_amd.kernels as K_
    real = K_.fused_nsf_chain_saved
    out = {}
    for chain in (True, False):
        for rep in range(2):
            K_.fused_nsf_chain_saved = real
            out[(chain, rep)] = t._step(model, x, chain, MP())
    K_.fused_nsf_chain_saved = real
    for k in [(True, 1), (False, 0), (False, 1)]:
        a, b = out[(True, 0)], out[k]
        dx = (a[4] - b[4]).abs().max().item()
        dp = max((a[5][n] - b[5][n]).abs().max().item() for n in a[5])
        print(rows, "chain0 vs", k, "x.grad maxdiff", dx, "param maxdiff", dp, "loss eq", torch.equal(a[1], b[1]))
