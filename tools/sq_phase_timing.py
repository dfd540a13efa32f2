"""Phase clocks of the sequential NSF_AR inverse (nfk_ar_seqinv) at
Polymer.yaml's shape (dim 2048, K 32, H 100, 40 rows): thread 0 of row 0's
finish workgroup and of the first layer-1 chunk workgroup stamp the shader
clock (nfk_debug_sq_timing), and this prints the mean cycles of each phase
over the columns.  Diagnostic only."""
import ctypes
import json
import sys

import torch

sys.path.insert(0, ".")
import nf.flows as nff  # noqa: E402
from normalizingflow_amd import kernels as K_  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    dim, H, rows = 2048, 100, 40
    torch.manual_seed(0)
    flow = nff.NSF_AR(dim=dim, K=32, B=0.5, hidden_dim=H).to(dev)
    z = torch.randn(rows, dim, device=dev) * 0.3
    lib = K_._lib.load()
    lib.nfk_debug_sq_timing.restype = ctypes.c_void_p
    lib.nfk_debug_sq_timing.argtypes = [ctypes.c_void_p]
    with torch.no_grad():
        flow.inverse(z)
        torch.cuda.synchronize()
        buf = torch.zeros(dim * 12, dtype=torch.int64, device=dev)
        lib.nfk_debug_sq_timing(ctypes.c_void_p(buf.data_ptr()))
        flow.inverse(z)
        torch.cuda.synchronize()
        lib.nfk_debug_sq_timing(None)
    t = buf.view(dim, 12).cpu().double()
    names = {"stage": (0, 1), "layer1": (1, 2), "layer2": (2, 3), "layer3": (3, 4), "spline": (4, 5),
             "stores": (5, 6), "finish_total": (0, 6), "chunk_stage": (8, 9), "chunk_gemm": (9, 10),
             "chunk_total": (8, 10), "chunk_start_vs_finish_start": (0, 8)}
    out = {}
    sel = slice(1, dim - 1)  # columns with both a finish and chunks
    for k, (a, b) in names.items():
        d = (t[sel, b] - t[sel, a])
        out[k] = {"mean": round(d.mean().item(), 1), "median": round(d.median().item(), 1)}
    # consecutive columns' finish starts: the whole per-column period in clocks
    st = t[1:dim, 0]
    per = (st[1:] - st[:-1])
    out["column_period"] = {"mean": round(per.mean().item(), 1), "median": round(per.median().item(), 1)}
    out["column0"] = {"spline": round((t[0, 5] - t[0, 4]).item(), 1), "total": round((t[0, 6] - t[0, 0]).item(), 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
