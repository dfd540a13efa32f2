"""wgrad forms at RealNVP's first layer (g [2^20, 100], h = x half [2^20, 32] of
a [2^20, 64] tensor) and layer 3 ([2^20, 32] vs [2^20, 101 (of 104)])."""
import time
import torch

B = 1 << 20
dev = torch.device("cuda:0")


def t(fn, n=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def split(g, h, S, trans):
    R = B // S
    if trans:
        return torch.bmm(h.view(S, R, -1).transpose(1, 2), g.view(S, R, -1)).sum(0).t()
    return torch.bmm(g.view(S, R, -1).transpose(1, 2), h.view(S, R, -1)).sum(0)


x = torch.randn(B, 64, device=dev)
cases = {
    "L1: g[B,100] h=x[:, :32] (ld 64)": (torch.randn(B, 100, device=dev), x[:, :32]),
    "L1: g[B,100] h=x[:, 32:] (ld 64)": (torch.randn(B, 100, device=dev), x[:, 32:]),
    "L3: g[B,32] h=[B,101] (ld 104)": (torch.randn(B, 32, device=dev), torch.randn(B, 104, device=dev)[:, :101]),
    "L2: g[B,100] h=[B,101] (ld 104)": (torch.randn(B, 100, device=dev), torch.randn(B, 104, device=dev)[:, :101]),
    "c3 L3: g[B,736] h=[B,101] (ld 104)": (torch.randn(B, 736, device=dev), torch.randn(B, 104, device=dev)[:, :101]),
}
for k, (g, h) in cases.items():
    for trans in (False, True):
        print("%-36s trans=%d %.3f ms" % (k, trans, t(lambda: split(g, h, 64, trans))), flush=True)
