"""Microbenchmark of the split-K weight-gradient GEMM (fcnn_grad.wgrad) at c3's
layer-3 shape: g [2^20, 736], h [2^20, 101 (of 104)]; variants of the split and
the operand order."""
import time
import torch

B, P, N = 1 << 20, 736, 101
dev = torch.device("cuda:0")
g = torch.randn(B, P, device=dev) * 1e-3
ha = torch.randn(B, 104, device=dev)
h = ha[:, :N]


def split(gm, hm, S, trans):
    R = B // S
    if trans:
        return torch.bmm(hm.view(S, R, -1).transpose(1, 2), gm.view(S, R, -1)).sum(0).t()
    return torch.bmm(gm.view(S, R, -1).transpose(1, 2), hm.view(S, R, -1)).sum(0)


def t(fn, n=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


ref = (g.double().t() @ h.double())
for S in (16, 32, 64, 128, 256):
    for trans in (False, True):
        ms = t(lambda: split(g, h, S, trans))
        err = float((split(g, h, S, trans).double() - ref).abs().max() / ref.abs().max())
        print("S=%4d trans=%d  %.3f ms  rel err %.2e" % (S, trans, ms, err), flush=True)
hc = h.contiguous()
for S in (64,):
    for trans in (False, True):
        print("contig h S=%d trans=%d %.3f ms" % (S, trans, t(lambda: split(g, hc, S, trans))), flush=True)
print("plain mm %.3f ms" % t(lambda: g.t() @ h))
