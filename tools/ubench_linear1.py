"""FCNN first-layer recompute y = x W1^T + b1 at c2's shape: x = one half of a
[2^20, 64] tensor ([2^20, 32], row stride 64), W1 [100, 32]."""
import time
import torch

B = 1 << 20
dev = torch.device("cuda:0")
x = torch.randn(B, 64, device=dev)
W = torch.randn(100, 32, device=dev) * 0.1
b = torch.randn(100, device=dev)


def t(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


for name, xin in (("x[:, :32] strided", x[:, :32]), ("x[:, 32:] strided", x[:, 32:]),
                  ("contiguous copy", x[:, :32].contiguous())):
    print("%-20s addmm %.3f ms" % (name, t(lambda: torch.addmm(b, xin, W.t()))), flush=True)
    print("%-20s copy+addmm %.3f ms" % (name, t(lambda: torch.addmm(b, xin.contiguous(), W.t()))), flush=True)
    print("%-20s (W x^T)^T %.3f ms" % (name, t(lambda: torch.addmm(b[:, None], W, xin.t()).t())), flush=True)
