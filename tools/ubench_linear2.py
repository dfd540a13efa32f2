"""The FCNN hidden layer y = h W^T + b at H = 100 (h [2^20, 100], W [100, 100]):
forms that lead hipBLASLt to different kernels."""
import time
import torch

B, H = 1 << 20, 100
dev = torch.device("cuda:0")
h = torch.tanh(torch.randn(B, H, device=dev))
W = torch.randn(H, H, device=dev) * 0.1
b = torch.randn(H, device=dev)
Wt = W.t().contiguous()
ha = torch.empty(B, 104, device=dev)
ha[:, :H] = h
hp = ha[:, :H]


def t(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


ref = torch.addmm(b, h, W.t())
forms = {
    "addmm(b, h, W.t())": lambda: torch.addmm(b, h, W.t()),
    "addmm(b, h, Wt)": lambda: torch.addmm(b, h, Wt),
    "mm(h, W.t()) + b": lambda: torch.mm(h, W.t()) + b,
    "mm(h, Wt) + b": lambda: torch.mm(h, Wt) + b,
    "addmm(b, hpad104, W.t())": lambda: torch.addmm(b, hp, W.t()),
    "addmm(b, hpad104, Wt)": lambda: torch.addmm(b, hp, Wt),
    "F.linear(h, W, b)": lambda: torch.nn.functional.linear(h, W, b),
    "(W h^T)^T + b": lambda: torch.addmm(b[:, None], W, h.t()).t(),
}
for k, f in forms.items():
    y = f()
    print("%-28s %.3f ms  max|d| %.2e" % (k, t(f), float((y - ref).abs().max())), flush=True)
