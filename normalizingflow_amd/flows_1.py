"""Layers of the reference's ``nf/flows_1.py``.

Every class there is the same as in ``nf/flows.py`` or ``flows_1``'s own
Planar / Radial / MAF / ActNorm / OneByOneConv (all in ``flows.py`` here),
except ``NSF_AR``: flows_1.py defines it three times and its last definition
(flows_1.py:395-465), which ``from nf.flows_1 import NSF_AR`` binds, is a
different layer from nf/flows.py's NSF_AR:

* ``periodic=True`` keyword; ``dim`` conditioner nets and no ``init_param``;
* net i reads the first i coordinates of the layer's INPUT (x in forward, z in
  inverse, flows_1.py:428-433 and 450-455) -- a zero column for i = 0 --
  mapped through cos/sin(pi v / B) when periodic (input width 2i, or 2 for
  i = 0; i, or 1, otherwise).

The spline of every coordinate runs through the same HIP kernels as
nf/flows.py's NSF_AR (trig features, conditioner FCNN, nfk_rqs_coupling).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.init as init

from . import fcnn_grad
from . import kernels as K_
from .flows import FCNN, _HipFlow, _dense, _is_stock_fcnn, _vjp_out
from .flows import MAF, ActNorm, NSF_CL, OneByOneConv, Planar, Radial, RealNVP  # noqa: F401
from .flows import functional_derivatives  # noqa: F401

__all__ = ["NSF_AR", "FCNN", "NSF_CL", "RealNVP", "Planar", "Radial", "MAF", "ActNorm",
           "OneByOneConv"]


class NSF_AR(_HipFlow):
    """Autoregressive neural-spline flow of nf/flows_1.py:395-465."""

    _torch_math = "nsf_ar_flows1"  # its differentiable restatement (not flows.NSF_AR's)

    def __init__(self, dim, K=32, B=3, hidden_dim=800, base_network=FCNN, device="cpu", periodic=True):
        super().__init__()
        self.dim = dim
        self.K = K
        self.B = B
        self.device = device
        self.periodic = periodic
        self.layers = nn.ModuleList()
        for i in range(dim):  # flows_1.py:407-417, same construction (and RNG) order
            width = (2 * i if i else 2) if periodic else (i if i else 1)
            self.layers += [base_network(width, 3 * K - 1, hidden_dim).to(self.device)]
        self._cols = {}

    @property
    def _n_status(self):
        return self.dim

    def reset_parameters(self):
        # flows_1.py:419-420 refers to an init_param this class never creates:
        # the reference raises AttributeError here, and so does this
        init.uniform_(self.init_param, -1 / 2, 1 / 2)

    def trig_transform(self, x):
        feat = torch.empty(x.shape[0], 2 * x.shape[1], dtype=torch.float32, device=x.device)
        K_.trig_features(x, feat, self.B)
        return feat

    def _col(self, i, device):
        key = (i, str(device))
        c = self._cols.get(key)
        if c is None:
            c = self._cols[key] = torch.tensor([i], dtype=torch.int32, device=device)
        return c

    def _run(self, x, inverse, logdet, mode, status):
        if x.shape[1] != self.dim:
            raise RuntimeError("NSF_AR(dim=%d) got %d features" % (self.dim, x.shape[1]))
        n = x.shape[0]
        z = torch.zeros_like(x, memory_format=torch.contiguous_format)
        b = float(self.B)
        zero_col = None
        for i in range(self.dim):
            if i == 0:
                zero_col = torch.zeros(n, 1, dtype=torch.float32, device=x.device)
                src = zero_col
            else:
                src = x[:, :i]  # the layer's input, in both directions
            feat = self.trig_transform(src) if self.periodic else src
            params = self.layers[i](feat).contiguous()
            m = mode if (i == 0 or mode == K_.MODE_NONE) else K_.MODE_ACC
            col = self._col(i, x.device)
            K_.rqs_coupling(x, params, col, col, z, logdet=logdet, logdet_mode=m, K=self.K,
                            left=-b, right=b, bottom=-b, top=b, tails=True, param_mode=0,
                            inverse=inverse,
                            status=None if status is None else status[i:i + 1])
        return z

    def _vjp(self, x, names, params, gz, gld, inverse, need):
        """Backward by hand for stock FCNN conditioners (else None: autograd
        recompute).  Every net reads the layer's input, so the columns are
        independent: per column the spline VJP (nfk_rqs_coupling_bwd), then the
        net's (fcnn_grad) and, when periodic, the trig features'
        (nfk_trig_features_bwd) into dL/dx[:, :i]; column 0's zero input
        column takes no gradient."""
        if not all(_is_stock_fcnn(n) for n in self.layers) or x.shape[1] != self.dim:
            return None
        p = {n: t.detach() for n, t in zip(names, params)}
        want = {n for n, r in zip(names, need[1:]) if r}
        x = x.detach()
        B, b = x.shape[0], float(self.B)
        gzc = _dense(gz, x)
        gldc = None if gld is None else gld.contiguous()
        gx = torch.empty_like(x)
        grads = {}
        for i in range(self.dim):
            src = torch.zeros(B, 1, dtype=torch.float32, device=x.device) if i == 0 else x[:, :i]
            feat = self.trig_transform(src) if self.periodic else src.contiguous()
            prm, cache = fcnn_grad.forward_saved(p, "layers.%d." % i, feat)
            gprm = torch.empty_like(prm)
            col = self._col(i, x.device)
            K_.rqs_coupling_bwd(x, prm, col, col, gzc, gldc, gprm, gx, K=self.K, left=-b, right=b,
                                bottom=-b, top=b, tails=True, param_mode=0, inverse=inverse)
            gfeat, gr = fcnn_grad.vjp(p, "layers.%d." % i, cache, gprm, i > 0, want)
            grads.update(gr)
            if i > 0:
                if self.periodic:
                    K_.trig_features_bwd(src, gfeat, gx, b)
                else:
                    gx[:, :i] += gfeat
        return _vjp_out(names, need, gx, grads)

    def forward(self, x):
        return self._call(x, False)

    def inverse(self, z):
        return self._call(z, True)
