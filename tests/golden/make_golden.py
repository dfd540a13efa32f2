"""Generate golden input/output vectors from the REFERENCE implementation.

Run in the build container (where /root/reference exists):

    python tests/golden/make_golden.py

It imports the reference's own ``nf`` package from /root/reference (read-only,
no bytecode written).  ``nf/utils.py:4`` imports MDAnalysis, which is not
installed and is never used by that file, so an empty module object stands in
for it.  Nothing else of the reference is altered.

Outputs ``tests/golden/<case>.npz`` (arrays only, loadable with
``allow_pickle=False``): inputs, the layer's state_dict (``sd.<key>``),
reference outputs in fp32 and, where meaningful, an fp64 companion run, plus
a JSON ``meta`` string with the constructor arguments.  The fixtures are data;
no reference source travels with them.
"""
from __future__ import annotations

import json
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

sys.dont_write_bytecode = True
# make sure OUR nf/ package cannot shadow the reference's namespace package
sys.path[:] = [p for p in sys.path if os.path.abspath(p or ".") not in (REPO, HERE)]
sys.path.insert(0, REF)
sys.modules.setdefault("MDAnalysis", types.ModuleType("MDAnalysis"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import nf.flows as rflows  # noqa: E402
import nf.flows_1 as rflows1  # noqa: E402
import nf.models as rmodels  # noqa: E402
import nf.utils as rutils  # noqa: E402

assert os.path.realpath(rflows.__file__).startswith(REF), rflows.__file__


def _np(t):
    return t.detach().cpu().numpy()


def _save(name, meta, arrays, module=None):
    out = {"meta": np.array(json.dumps(meta))}
    for k, v in arrays.items():
        out[k] = _np(v) if torch.is_tensor(v) else np.asarray(v)
    if module is not None:
        for k, v in module.state_dict().items():
            out["sd." + k] = _np(v)
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print("wrote", path, sum(a.nbytes for a in out.values()), "bytes")


def _f64(module):
    import copy
    return copy.deepcopy(module).double()


# ---------------------------------------------------------------- raw spline
def case_rqs(name, n, K, scale, tail, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, generator=g) * 2.0
    x[:8] = torch.tensor([-tail, tail, -tail - 1e-3, tail + 1e-3, 0.0, 1e-7, -4 * tail, 4 * tail])
    uw = torch.randn(n, K, generator=g) * scale
    uh = torch.randn(n, K, generator=g) * scale
    ud = torch.randn(n, K - 1, generator=g) * scale
    arrays = dict(x=x, uw=uw, uh=uh, ud=ud)
    y, lad = rutils.unconstrained_RQS(x.clone(), uw.clone(), uh.clone(), ud.clone(),
                                      inverse=False, tail_bound=tail)
    arrays.update(y=y, lad=lad)
    yi, ladi = rutils.unconstrained_RQS(y.clone(), uw.clone(), uh.clone(), ud.clone(),
                                        inverse=True, tail_bound=tail)
    arrays.update(inv_y=yi, inv_lad=ladi)
    y64, lad64 = rutils.unconstrained_RQS(x.double(), uw.double(), uh.double(), ud.double(),
                                          inverse=False, tail_bound=tail)
    arrays.update(y_f64=y64, lad_f64=lad64)
    _save(name, dict(kind="rqs", K=K, tail_bound=tail, scale=scale, seed=seed), arrays)


# ---------------------------------------------------------------- layers
def case_layer(name, ctor, kwargs, x, inverse=True, f64=True, init=None, seed=1234):
    torch.manual_seed(seed)
    layer = ctor(**kwargs)
    if init is not None:
        init(layer)
    arrays = dict(x=x)
    with torch.no_grad():
        z, ld = layer.forward(x.clone())
        arrays.update(z=z, ld=ld)
        if inverse:
            xi, ldi = layer.inverse(z.clone())
            arrays.update(rt_x=xi, rt_ld=ldi)
            xa, lda = layer.inverse(x.clone())
            arrays.update(inv_x=xa, inv_ld=lda)
        if f64:
            l64 = _f64(layer)
            z64, ld64 = l64.forward(x.double())
            arrays.update(z_f64=z64, ld_f64=ld64)
    meta = dict(kind="layer", type=ctor.__name__, kwargs={k: v for k, v in kwargs.items()
                                                         if k not in ("nonlinearity",)},
                seed=seed)
    if "nonlinearity" in kwargs:
        meta["nonlinearity"] = kwargs["nonlinearity"].__name__
    _save(name, meta, arrays, layer)


def case_onebyone(name, dim, x, seed=1234):
    """OneByOneConv: P, L, S, U from np.random (flows_1.py:227-233); a fresh
    instance per inverse call (the reference caches W^-1 once)."""
    def make():
        np.random.seed(seed)
        torch.manual_seed(seed)
        return rflows1.OneByOneConv(dim)
    layer = make()
    arrays = dict(x=x)
    with torch.no_grad():
        z, ld = layer.forward(x.clone())
        arrays.update(z=z, ld=ld)
        xi, ldi = layer.inverse(z.clone())
        arrays.update(rt_x=xi, rt_ld=ldi)
        xa, lda = make().inverse(x.clone())
        arrays.update(inv_x=xa, inv_ld=lda)
    _extra_p(layer, arrays)
    _save(name, dict(kind="layer", type="OneByOneConv", kwargs=dict(dim=dim), seed=seed,
                     np_seed=seed), arrays, layer)


def actnorm_init(layer):
    with torch.no_grad():
        g = torch.Generator().manual_seed(9)
        layer.mu.copy_(torch.randn(layer.dim, generator=g) * 0.5)
        layer.log_sigma.copy_(torch.randn(layer.dim, generator=g) * 0.3)


def radial_init(layer):
    with torch.no_grad():
        g = torch.Generator().manual_seed(7)
        layer.x0.copy_(torch.randn(layer.x0.shape, generator=g) * 0.3)
        layer.log_alpha.fill_(0.1)
        layer.beta.fill_(0.5)


# ---------------------------------------------------------------- models
def _extra_p(module, arrays):
    """OneByOneConv keeps its permutation P outside the state_dict
    (flows_1.py:229): save it as sd.<prefix>P so the fixture is complete."""
    for name, m in module.named_modules():
        if type(m).__name__ == "OneByOneConv":
            arrays["sd." + (name + "." if name else "") + "P"] = m.P


def case_model(name, flow_specs, dim, var, n, seed=1234, init=None):
    import copy
    torch.manual_seed(seed)
    np.random.seed(seed)
    flows = [ctor(**kw) for ctor, kw in flow_specs]
    if init is not None:
        init(flows)
    prior = torch.distributions.MultivariateNormal(torch.zeros(dim), var * torch.eye(dim))
    model = rmodels.NormalizingFlowModel(prior, flows)
    # OneByOneConv caches W^-1 once and raises on a second inverse (flows_1.py:244):
    # sample() runs on a fresh copy
    model_s = copy.deepcopy(model)
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(n, dim, generator=g) * 1.3
    arrays = dict(x=x)
    _extra_p(model, arrays)
    with torch.no_grad():
        z, plp, ld = model(x.clone())
        arrays.update(z=z, prior_lp=plp, ld=ld, log_prob=model.evaluate(x.clone()))
        try:
            xi, ldi = model.inverse(z.clone())
            arrays.update(rt_x=xi, rt_ld=ldi)
            torch.manual_seed(seed + 2)
            xs, lps, zs = model_s.sample(n)
            arrays.update(sample_x=xs, sample_log_px=lps, sample_z=zs)
        except NotImplementedError:  # Planar / Radial have no inverse
            pass
    _save(name, dict(kind="model", dim=dim, var=var, seed=seed,
                     layers=[dict(type=c.__name__, kwargs=kw) for c, kw in flow_specs]),
          arrays, model)


def extra_cases():
    """flows_1.py MAF / ActNorm / OneByOneConv."""
    g = torch.Generator().manual_seed(4242)
    x8 = torch.randn(256, 8, generator=g) * 1.3
    case_layer("maf_d8_h8", rflows1.MAF, dict(dim=8, hidden_dim=8), x8)
    x5 = torch.randn(128, 5, generator=g)
    case_layer("maf_d5_h16", rflows1.MAF, dict(dim=5, hidden_dim=16), x5)
    case_layer("actnorm_d8", rflows1.ActNorm, dict(dim=8), x8, init=actnorm_init)
    case_onebyone("onebyone_d8", 8, x8)
    case_onebyone("onebyone_d16", 16, torch.randn(128, 16, generator=g))

    def init_glow(flows):
        actnorm_init(flows[0])
    case_model("model_glow", [
        (rflows1.ActNorm, dict(dim=8)),
        (rflows1.OneByOneConv, dict(dim=8)),
        (rflows.NSF_CL, dict(size=4, dim=2, K=6, B=3, hidden_dim=16, mask=[0])),
        (rflows1.MAF, dict(dim=8, hidden_dim=8)),
        (rflows.RealNVP, dict(dim=8, hidden_dim=16))], dim=8, var=1.0, n=128, init=init_glow)


def main():
    g = torch.Generator().manual_seed(42)
    case_rqs("rqs_k4", 512, 4, 1.0, 3.0, 11)
    case_rqs("rqs_k8_extreme", 512, 8, 3.0, 3.0, 12)
    case_rqs("rqs_k16_tb1", 512, 16, 1.5, 1.0, 13)

    x8 = torch.randn(256, 8, generator=g) * 1.5
    case_layer("nsfcl_s4d2_k4_m0", rflows.NSF_CL,
               dict(size=4, dim=2, K=4, B=3, hidden_dim=16, mask=[0]), x8)
    case_layer("nsfcl_s4d2_k8_m1", rflows.NSF_CL,
               dict(size=4, dim=2, K=8, B=3, hidden_dim=16, mask=[1]), x8)
    x9 = torch.randn(128, 9, generator=g) * 1.2
    case_layer("nsfcl_s3d3_k5_m01", rflows.NSF_CL,
               dict(size=3, dim=3, K=5, B=2.5, hidden_dim=12, mask=[0, 1]), x9)
    case_layer("nsfcl_s3d3_k5_m12", rflows.NSF_CL,
               dict(size=3, dim=3, K=5, B=2.5, hidden_dim=12, mask=[1, 2]), x9)
    case_layer("nsfcl_s3d3_k10_m2", rflows.NSF_CL,
               dict(size=3, dim=3, K=10, B=2.0, hidden_dim=12, mask=[2]), x9)
    x64 = torch.randn(64, 64, generator=g)
    case_layer("nsfcl_c3_m1", rflows.NSF_CL,
               dict(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[1]), x64)

    x2 = torch.randn(256, 2, generator=g)
    case_layer("realnvp_d2", rflows.RealNVP, dict(dim=2, hidden_dim=16), x2)
    case_layer("realnvp_d8", rflows.RealNVP, dict(dim=8, hidden_dim=16), x8)

    for nl in (torch.tanh, F.leaky_relu, F.elu):
        case_layer("planar_d8_" + nl.__name__, rflows1.Planar, dict(dim=8, nonlinearity=nl), x8,
                   inverse=False)
    case_layer("radial_d8", rflows1.Radial, dict(dim=8), x8, inverse=False, init=radial_init)

    x4 = torch.randn(128, 4, generator=g) * 1.3
    case_layer("nsfar_d4_k4", rflows.NSF_AR, dict(dim=4, K=4, B=3, hidden_dim=16), x4)

    case_model("model_nsfcl4", [
        (rflows.NSF_CL, dict(size=4, dim=2, K=8, B=3, hidden_dim=16, mask=m))
        for m in ([0], [1], [0], [1])], dim=8, var=1.0, n=128)
    case_model("model_mixed", [
        (rflows.RealNVP, dict(dim=8, hidden_dim=16)),
        (rflows.NSF_CL, dict(size=4, dim=2, K=6, B=3, hidden_dim=16, mask=[0])),
        (rflows.NSF_CL, dict(size=4, dim=2, K=6, B=3, hidden_dim=16, mask=[1])),
        (rflows1.Planar, dict(dim=8))], dim=8, var=2.0, n=128)
    case_model("model_realnvp_c1", [(rflows.RealNVP, dict(dim=2, hidden_dim=32))
                                    for _ in range(4)], dim=2, var=1.0, n=256)


if __name__ == "__main__":
    if sys.argv[1:] == ["extra"]:
        extra_cases()
    else:
        main()
        extra_cases()
