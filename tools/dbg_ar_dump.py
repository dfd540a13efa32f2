"""Diagnostic (NFK_AR_DIAG_DUMP builds): conditioner 1's layer-1 / layer-2
activations and logits from the fused NSF_AR kernel vs the oracle's, per
hidden feature, for the first 64 rows."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nf.flows as nff  # noqa: E402
from normalizingflow_amd import _lib, config  # noqa: E402

dev = torch.device("cuda", 0)
config.STRICT_CHECKS = False
lib = _lib.load()
for H in [int(v) for v in os.environ.get("DBG_HS", "192,224").split(",")]:
    torch.manual_seed(5)
    layer = nff.NSF_AR(dim=2, K=32, B=1.462, hidden_dim=H)
    sd = {k: v.detach().double() for k, v in layer.state_dict().items()}
    x = torch.randn(64, 2, generator=torch.Generator().manual_seed(1)) * 0.9
    for rep in range(2):
        layer = layer.to(dev)
        with torch.no_grad():
            layer(x.to(dev))
        torch.cuda.synchronize()
        buf = np.zeros(3 * 64 * 512, dtype=np.float32)
        assert lib.nfk_ar_dbg_copy(buf.ctypes.data_as(ctypes.c_void_p)) == 0
        buf = buf.reshape(3, 64, 512)
        f = torch.cat((torch.cos(np.pi * x[:, :1].double() / 1.462), torch.sin(np.pi * x[:, :1].double() / 1.462)), 1)
        h1 = torch.tanh(f @ sd["layers.0.network.0.weight"].T + sd["layers.0.network.0.bias"])
        h2 = torch.tanh(h1 @ sd["layers.0.network.2.weight"].T + sd["layers.0.network.2.bias"])
        o = h2 @ sd["layers.0.network.4.weight"].T + sd["layers.0.network.4.bias"]
        for st, ref, n in ((0, h1, H), (1, h2, H), (2, o, 95)):
            got = torch.from_numpy(buf[st, :, :n]).double()
            err = (got - ref).abs()
            bad = (err > 1e-4).nonzero()
            print("H %d rep %d stage %d: max err %.3g; bad (row, feature) count %d, rows %s, features %s" % (
                H, rep, st, float(err.max()), bad.shape[0], sorted(set(bad[:, 0].tolist()))[:12],
                sorted(set(bad[:, 1].tolist()))[:24]), flush=True)
