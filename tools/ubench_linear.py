"""Forms of the FCNN output-layer recompute y = h W^T + b at c2's shape
(h [2^20, 100], W [32, 100]) through hipBLASLt."""
import time
import torch

B, H, O = 1 << 20, 100, 32
dev = torch.device("cuda:0")
ha = torch.randn(B, 104, device=dev)
h_str = ha[:, :H]
h_con = h_str.contiguous()
W = torch.randn(O, H, device=dev) * 0.1
b = torch.randn(O, device=dev)
Wt = W.t().contiguous()


def t(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


ref = torch.addmm(b, h_con, W.t())
forms = {
    "addmm(b, h_strided, W.t())": lambda: torch.addmm(b, h_str, W.t()),
    "addmm(b, h_contig, W.t())": lambda: torch.addmm(b, h_con, W.t()),
    "addmm(b, h_strided, Wt_contig)": lambda: torch.addmm(b, h_str, Wt),
    "addmm(b, h_contig, Wt_contig)": lambda: torch.addmm(b, h_con, Wt),
    "(W @ h_strided.t()).t() + b": lambda: torch.addmm(b[:, None], W, h_str.t()).t(),
    "F.linear(h_strided, W, b)": lambda: torch.nn.functional.linear(h_str, W, b),
}
for k, f in forms.items():
    y = f()
    err = float((y - ref).abs().max())
    print("%-34s %.3f ms  max|d| %.2e" % (k, t(f), err), flush=True)
