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
def case_layer(name, ctor, kwargs, x, inverse=True, f64=True, init=None, seed=1234, type_name=None):
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
    meta = dict(kind="layer", type=type_name or ctor.__name__, kwargs={k: v for k, v in kwargs.items()
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


# ------------------------------------------------- negative discriminant (utils.py:121)
def _knot_stack(u, K, tb):
    """The cumulative knots RQS builds from unnormalised logits u (utils.py:73-91
    op for op: softmax, floor, padded cumsum, affine map, pinned ends), used
    only to place inputs a few ulps below a bin's top knot."""
    w = torch.softmax(u, dim=-1)
    w = 1e-3 + (1 - 1e-3 * K) * w
    c = F.pad(torch.cumsum(w, dim=-1), pad=(1, 0), mode="constant", value=0.0)
    c = 2 * tb * c - tb
    c[..., 0] = -tb
    c[..., -1] = tb
    return c


def _below(v, j):
    """v stepped down by j[i] ulps (fp32), elementwise."""
    out = v.clone()
    for i in range(v.shape[0]):
        for _ in range(int(j[i])):
            out[i] = torch.nextafter(out[i], torch.tensor(-1e30))
    return out


def _asserts(fn):
    try:
        fn()
    except AssertionError:
        return True
    return False


def negdisc_cases():
    """Inputs for which the reference's inverse hits `assert (discriminant >=
    0).all()` (utils.py:121): fp32 cancellation in b^2 - 4ac when the input
    sits a few ulps below the top knot of a bin whose slope delta = h/w is
    huge.  Three fixtures: raw unconstrained_RQS (min derivative 1e-3, random
    extreme logits), one NSF_CL layer and a 2-layer NSF_CL model (B=6, so the
    double softmax of NSF_CL still reaches delta ~ e^12; the last FCNN layer
    has zero weights and a crafted bias, so every row has the same knots)."""
    K, tb, n = 8, 3.0, 4096
    g = torch.Generator().manual_seed(77)
    uw = torch.randn(n, K, generator=g) * 6
    uh = torch.randn(n, K, generator=g) * 6
    ud = torch.full((n, K - 1), -30.0) + torch.randn(n, K - 1, generator=g)
    cw, ch = _knot_stack(uw, K, tb), _knot_stack(uh, K, tb)
    kb = ((ch[:, 1:] - ch[:, :-1]) / (cw[:, 1:] - cw[:, :-1])).argmax(1)
    top = ch.gather(1, (kb + 1)[:, None])[:, 0]
    x = _below(top, torch.randint(1, 6, (n,), generator=g))
    ok = _asserts(lambda: rutils.unconstrained_RQS(x.clone(), uw.clone(), uh.clone(), ud.clone(),
                                                   inverse=True, tail_bound=tb))
    row_neg = [i for i in range(n) if _asserts(lambda: rutils.unconstrained_RQS(
        x[i:i + 1].clone(), uw[i:i + 1].clone(), uh[i:i + 1].clone(), ud[i:i + 1].clone(),
        inverse=True, tail_bound=tb))]
    assert ok and row_neg, "reference did not assert"
    _save("err_rqs_negdisc", dict(kind="negdisc_rqs", K=K, tail_bound=tb, seed=77),
          dict(x=x, uw=uw, uh=uh, ud=ud, ref_asserts=np.array(ok),
               row_neg=np.array(row_neg, dtype=np.int64)))

    # NSF_CL layer and model: a diverged conditioner (one NaN weight in the
    # output layer of psi).  The reference's forward then yields NaN for the
    # coordinate whose logit is NaN (and its row's log|det|), and its inverse
    # fails the same assert (NaN >= 0 is false).  A genuinely negative fp32
    # discriminant is ~5e-4 rare under NSF_CL's double softmax (slopes capped
    # near 1/min_bin_width, interior derivatives >= 0.69), so it cannot be
    # pinned robustly there; the raw case above pins it.
    size = 32
    gz = torch.Generator().manual_seed(78)
    x = torch.randn(512, 2 * size, generator=gz) * 1.2

    def poison(layer, row):
        with torch.no_grad():
            layer.psi.network[4].weight[row, 3] = float("nan")

    torch.manual_seed(1234)
    layer = rflows.NSF_CL(size=size, dim=2, K=8, B=3, hidden_dim=100, mask=[1])
    poison(layer, 5 * 23 + 2)      # W logit 2 of upper coordinate 5
    with torch.no_grad():
        z, ld = layer.forward(x.clone())
        ok = _asserts(lambda: layer.inverse(x.clone()))
    assert ok, "reference NSF_CL.inverse did not assert"
    _save("err_nsfcl_nan", dict(kind="nan_layer", type="NSF_CL",
                            kwargs=dict(size=size, dim=2, K=8, B=3, hidden_dim=100, mask=[1]),
                            seed=1234, nan_weight=[5 * 23 + 2, 3]),
          dict(x=x, z=z, ld=ld, inv_asserts=np.array(ok)), layer)

    torch.manual_seed(1234)
    flows = [rflows.NSF_CL(size=size, dim=2, K=8, B=3, hidden_dim=100, mask=[i % 2])
             for i in range(2)]
    poison(flows[1], 17 * 23 + 9)  # H logit 1 of upper coordinate 17 of the last layer
    prior = torch.distributions.MultivariateNormal(torch.zeros(2 * size), torch.eye(2 * size))
    model = rmodels.NormalizingFlowModel(prior, flows)
    def raised(fn):
        try:
            fn()
        except Exception as e:  # noqa: BLE001 -- record which error the reference raises
            return type(e).__name__
        return ""

    with torch.no_grad():
        # layer by layer (the model's own forward stops at the prior's
        # argument validation: ValueError on a NaN z, torch MultivariateNormal)
        zl, ld0 = flows[0].forward(x.clone())
        zm, ld1 = flows[1].forward(zl.clone())
        fwd_err = raised(lambda: model(x.clone()))
        eval_err = raised(lambda: model.evaluate(x.clone()))
        inv_err = raised(lambda: model.inverse(x.clone()))
    assert fwd_err == "ValueError" and eval_err == "ValueError" and inv_err == "AssertionError", \
        (fwd_err, eval_err, inv_err)
    _save("err_model_nan", dict(kind="nan_model", dim=2 * size, var=1.0, seed=1234,
                            layers=[dict(type="NSF_CL", kwargs=dict(size=size, dim=2, K=8, B=3,
                                                                    hidden_dim=100, mask=[i % 2]))
                                    for i in range(2)],
                            forward_raises=fwd_err, evaluate_raises=eval_err,
                            inverse_raises=inv_err),
          dict(x=x, z=zm, ld=ld0 + ld1), model)


def flows1_cases():
    """nf/flows_1.py's own NSF_AR (its last definition, flows_1.py:395-465),
    which `from nf.flows_1 import NSF_AR` binds: periodic and plain inputs (no fp64
    companion: its i = 0 input is an fp32 zeros column, flows_1.py:430)."""
    g = torch.Generator().manual_seed(4343)
    x4 = torch.randn(128, 4, generator=g) * 1.3
    case_layer("nsfar1_d4_k4_periodic", rflows1.NSF_AR, dict(dim=4, K=4, B=3, hidden_dim=16), x4, f64=False,
               type_name="NSF_AR_flows1")
    x3 = torch.randn(128, 3, generator=g) * 1.3
    case_layer("nsfar1_d3_k5_plain", rflows1.NSF_AR,
               dict(dim=3, K=5, B=2.5, hidden_dim=12, periodic=False), x3, f64=False,
               type_name="NSF_AR_flows1")


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


def _steep_nsfcl(B, size, K, mask, seed):
    """An NSF_CL layer whose psi output layer has zero weights and a crafted
    bias, so every row shares knots that make one bin per upper coordinate as
    steep as NSF_CL's double softmax allows (width at the 1e-3 floor, height
    ~1 - K 1e-3 of the range: slope ~990) with the smallest interior knot
    derivative (softplus(softplus(-30)) + 1e-3 = 0.694) at its top.  Returns
    (layer, top): top[j] = the fp32 top knot (in y) of coordinate j's steep bin."""
    g = torch.Generator().manual_seed(seed)
    torch.manual_seed(seed)
    layer = rflows.NSF_CL(size=size, dim=2, K=K, B=B, hidden_dim=16, mask=mask)
    n_up = size
    bias = torch.zeros(n_up, 3 * K - 1)
    ks = []
    for j in range(n_up):
        k = j % (K - 1)                  # an interior top knot k + 1
        m = (k + 2 + j // (K - 1)) % K   # the widest-bin of the x knots (never k)
        m = m if m != k else (k + 1) % K
        uw = torch.randn(K, generator=g)
        uw[m] = 40.0
        uh = torch.randn(K, generator=g)
        uh[k] = 40.0
        bias[j] = torch.cat([uw, uh, torch.full((K - 1,), -30.0)])
        ks.append(k)
    with torch.no_grad():
        layer.psi.network[4].weight.zero_()
        layer.psi.network[4].bias.copy_(bias.reshape(-1))
    ch = _knot_stack(2 * B * torch.softmax(bias[:, K:2 * K], dim=-1), K, B)
    top = torch.stack([ch[j, ks[j] + 1] for j in range(n_up)])
    return layer, top


def negdisc_cl_cases():
    """NSF_CL inputs on the knife edge of utils.py:121's assert.
    At the top knot y_k+1 of a bin the exact discriminant is (h d_k+1)^2, a
    fraction (d_k+1 / 2 delta)^2 ~ 1.2e-7 of b^2 at NSF_CL's steepest bins
    (the double softmax caps delta = h / w near 990, interior derivatives are
    >= 0.694): one or two fp32 ulps.  The fixture puts every upper coordinate
    of 1,024 rows 0-5 ulps under such a top knot (8,192 knife-edge elements)
    and records what the reference does -- its inverse (layer and 2-layer
    model) and the fp64 truth."""
    K, B, size = 8, 6.0, 8
    g = torch.Generator().manual_seed(91)
    layer, top = _steep_nsfcl(B, size, K, [0], 91)
    n = 1024
    x = torch.randn(n, 2 * size, generator=g)
    ulps = torch.randint(0, 6, (n, size), generator=g)
    for j in range(size):
        x[:, 2 * j + 1] = _below(top[j].expand(n).clone(), ulps[:, j] + 1)
    with torch.no_grad():
        asserts = _asserts(lambda: layer.inverse(x.clone()))
        row_asserts = [i for i in range(n) if _asserts(lambda: layer.inverse(x[i:i + 1].clone()))]
        xi, ldi = (None, None) if asserts else layer.inverse(x.clone())
        x64, ld64 = _f64(layer).inverse(x.double())
    arrays = dict(x=x, ulps=ulps, ref_asserts=np.array(asserts), row_asserts=np.array(row_asserts, dtype=np.int64),
                  inv_x_f64=x64, inv_ld_f64=ld64)
    if xi is not None:
        arrays.update(inv_x=xi, inv_ld=ldi)
    _save("negdisc_nsfcl_edge", dict(kind="negdisc_edge", type="NSF_CL",
                                     kwargs=dict(size=size, dim=2, K=K, B=B, hidden_dim=16, mask=[0]),
                                     seed=91), arrays, layer)
    print("layer: reference asserts on %d of %d knife-edge rows" % (len(row_asserts), n))

    # 2-layer model (a chained launch in inference): the last layer (mask [1],
    # the first inverted) steep on the knife edge, the first steep as well
    l0, _ = _steep_nsfcl(B, size, K, [0], 92)
    l1, top1 = _steep_nsfcl(B, size, K, [1], 93)
    prior = torch.distributions.MultivariateNormal(torch.zeros(2 * size), torch.eye(2 * size))
    model = rmodels.NormalizingFlowModel(prior, [l0, l1])
    z = torch.randn(n, 2 * size, generator=g)
    ulps1 = torch.randint(0, 6, (n, size), generator=g)
    for j in range(size):  # mask [1]: the upper coordinate of particle j is column 2 j
        z[:, 2 * j] = _below(top1[j].expand(n).clone(), ulps1[:, j] + 1)
    with torch.no_grad():
        m_asserts = _asserts(lambda: model.inverse(z.clone()))
        m_rows = [i for i in range(n) if _asserts(lambda: model.inverse(z[i:i + 1].clone()))]
        xm, ldm = (None, None) if m_asserts else model.inverse(z.clone())
        xm64, ldm64 = _f64(model).inverse(z.double())
    arrays = dict(z=z, ulps=ulps1, ref_asserts=np.array(m_asserts), row_asserts=np.array(m_rows, dtype=np.int64),
                  inv_x_f64=xm64, inv_ld_f64=ldm64)
    if xm is not None:
        arrays.update(inv_x=xm, inv_ld=ldm)
    _save("negdisc_model_edge", dict(kind="negdisc_edge_model", dim=2 * size, var=1.0, seed=92,
                                     layers=[dict(type="NSF_CL", kwargs=dict(size=size, dim=2, K=K, B=B,
                                                                              hidden_dim=16, mask=mk))
                                             for mk in ([0], [1])]), arrays, model)
    print("model: reference asserts on %d of %d knife-edge rows" % (len(m_rows), n))


def _f64_run(layer, inputs):
    """The fp64 companion of a layer's forward / inverse outputs:
    {"<out>_f64", "<ld>_f64"} for each (out name -> input) of ``inputs``
    ("z": forward of the input, anything else: inverse).  Run with fp64 as
    torch's default dtype, so the reference's own log_det accumulator
    (``torch.zeros(z.shape[0])``, flows.py:177, 195) is fp64 too: the
    companion is then the fp64 truth of the sum over every column, not an
    fp32 sum of fp64 terms.  (trig_transform's ``torch.tensor(np.pi)``,
    flows.py:173, is then fp64 as well; the fp32 pi moves log|det| by < 1e-8
    at these shapes.)"""
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        l64 = _f64(layer)
        out = {}
        with torch.no_grad():
            for name, v in inputs.items():
                fn = l64.forward if name == "z" else l64.inverse
                o, ld = fn(v.double().clone())
                assert o.dtype == torch.float64 and ld.dtype == torch.float64
                ldname = {"z": "ld", "rt_x": "rt_ld", "inv_x": "inv_ld"}[name]
                out.update({name + "_f64": o, ldname + "_f64": ld})
        return out
    finally:
        torch.set_default_dtype(prev)


def case_layer_seeded(name, ctor, kwargs, x, seed=1234):
    """case_layer for a layer too large to commit its weights (the
    applications' NSF_AR: 18 M parameters): the fixture holds the seed and, per
    state_dict entry, the fp64 sum, the fp64 sum of squares and the first 8
    values; tests/golden_io.py rebuilds the weights from the seed through the
    package's own constructor (same init order as the reference) and checks
    them against these before use.  With fp64 companions of the forward and
    both inverses (_f64_run), so a test can tell the reference's own fp32
    error from ours."""
    torch.manual_seed(seed)
    layer = ctor(**kwargs)
    arrays = dict(x=x)
    with torch.no_grad():
        z, ld = layer.forward(x.clone())
        arrays.update(z=z, ld=ld)
        xi, ldi = layer.inverse(z.clone())
        arrays.update(rt_x=xi, rt_ld=ldi)
        xa, lda = layer.inverse(x.clone())
        arrays.update(inv_x=xa, inv_ld=lda)
    arrays.update(_f64_run(layer, dict(z=x, rt_x=z, inv_x=x)))
    sd = layer.state_dict()
    sums = [torch.stack([v.detach().double().flatten().sum(), v.detach().double().flatten().square().sum()])
            for v in sd.values()]
    heads = [torch.nn.functional.pad(v.detach().flatten()[:8], (0, max(0, 8 - v.numel()))) for v in sd.values()]
    meta = dict(kind="layer", type=ctor.__name__, kwargs=kwargs, seed=seed, sd_from_seed=True)
    if len(sd) > 1000:
        # thousands of tensors (Polymer's 2,047 conditioners): one array each of
        # sums and heads in state_dict order (per-entry arrays cost ~0.5 KB of
        # zip headers apiece)
        arrays["sdsum_all"] = torch.stack(sums)
        arrays["sdhead_all"] = torch.stack(heads)
        meta["sd_keys"] = list(sd.keys())
        meta["sd_numel"] = [int(v.numel()) for v in sd.values()]
    else:
        for (k, v), sm in zip(sd.items(), sums):
            arrays["sdsum." + k] = sm
            arrays["sdhead." + k] = v.detach().flatten()[:8].clone()
    _save(name, meta, arrays)


def ar_cases():
    """NSF_AR at the shapes of the fused layer kernel (nfk_fused_ar): the
    applications' Gaussian.yaml flow (nparticles 20 x dim 2 = 40 coordinates,
    nsplines 10, hidden 80, B = ncellx * cell_len / 2 = 4, setup.py:42-58) and
    config.py's defaults (nsplines 32, hidden 100) at 24 coordinates."""
    g = torch.Generator().manual_seed(31)
    x40 = torch.randn(96, 40, generator=g) * 1.5
    case_layer("nsfar_d40_k10_h80", rflows.NSF_AR, dict(dim=40, K=10, B=4.0, hidden_dim=80), x40)
    x24 = torch.randn(64, 24, generator=g) * 1.2
    case_layer("nsfar_d24_k32_h100", rflows.NSF_AR, dict(dim=24, K=32, B=3, hidden_dim=100), x24)


def ar_app_cases():
    """NSF_AR at the applications' own shape: Einstein.yaml / LJ.yaml (flow
    NSF_AR, nsplines 32, hidden_dim 354; nparticles 32 x dim 3 = 96
    coordinates, setup.py:48, 57-58), B = (nparticles / (8 rho))^(1/3) at
    Einstein's rho 1.28 (setup.py:42-43); positions inside the box mostly.
    (Fe_*.yaml's 54 particles, dim 162, are ar_fe_cases.)"""
    B = (32 / (8 * 1.28)) ** (1.0 / 3.0)
    g = torch.Generator().manual_seed(37)
    x = torch.randn(64, 96, generator=g) * (0.6 * B)
    case_layer_seeded("nsfar_d96_k32_h354", rflows.NSF_AR, dict(dim=96, K=32, B=B, hidden_dim=354), x)


def ar_fe_cases():
    """NSF_AR at the Fe configs' shape (applications/input/Fe_100K.yaml:8,18-20;
    Fe_400K / Fe_700K the same): nparticles 54 x dim 3 (config.py:14) = 162
    coordinates (setup.py:48), nsplines 32, hidden_dim 354, B = ncellx *
    cell_len / 2 = 3 * 2.8841 / 2 (setup.py:44-45), at the configs' training
    batch of 50 rows (Fe_*.yaml batch_size)."""
    B = 3 * 2.8841 / 2
    g = torch.Generator().manual_seed(41)
    x = torch.randn(50, 162, generator=g) * (0.6 * B)
    case_layer_seeded("nsfar_d162_k32_h354", rflows.NSF_AR, dict(dim=162, K=32, B=B, hidden_dim=354), x)


def ar_polymer_cases():
    """NSF_AR at Polymer.yaml's shape (applications/input/Polymer.yaml:8-9,
    17-18): nparticles 2048 x dim 1 = 2048 coordinates, nsplines 32,
    hidden_dim commented out (:21) so config.py:40's 100, B = ncellx *
    cell_len / 2 = 0.5, at the config's 40-row batch.  2,047 conditioners
    FCNN(2i, 95, 100): 0.42 G weights, rebuilt from the seed."""
    g = torch.Generator().manual_seed(43)
    x = torch.randn(40, 2048, generator=g) * 0.3
    case_layer_seeded("nsfar_d2048_k32_h100", rflows.NSF_AR, dict(dim=2048, K=32, B=0.5, hidden_dim=100), x)


def rnvp_polymer_cases():
    """RealNVP at Polymer_rnvp.yaml's shape (applications/input/Polymer_rnvp.yaml:
    8-9, 16-18: nparticles 2048 x dim 1, RealNVP with hidden_dim 4000; the
    driver applications/examples/polymer.py:29 loads this config) at the
    config's 40-row batch (:30).  Four FCNN(1024, 1024, 4000) conditioners,
    96.8 M parameters: rebuilt from the seed.  Inputs at the prior's scale
    (vars 0.1, :24)."""
    g = torch.Generator().manual_seed(47)
    x = torch.randn(40, 2048, generator=g) * 0.1 ** 0.5
    case_layer_seeded("realnvp_d2048_h4000", rflows.RealNVP, dict(dim=2048, hidden_dim=4000), x)


if __name__ == "__main__":
    if sys.argv[1:] == ["rnvp_polymer"]:
        rnvp_polymer_cases()
    elif sys.argv[1:] == ["ar_fe"]:
        ar_fe_cases()
    elif sys.argv[1:] == ["ar_polymer"]:
        ar_polymer_cases()
    elif sys.argv[1:] == ["ar"]:
        ar_cases()
    elif sys.argv[1:] == ["ar_app"]:
        ar_app_cases()
    elif sys.argv[1:] == ["negdisc_cl"]:
        negdisc_cl_cases()
    elif sys.argv[1:] == ["extra"]:
        extra_cases()
    elif sys.argv[1:] == ["negdisc"]:
        negdisc_cases()
    elif sys.argv[1:] == ["flows1"]:
        flows1_cases()
    else:
        main()
        extra_cases()
        ar_cases()
        negdisc_cl_cases()
        negdisc_cases()
        flows1_cases()
