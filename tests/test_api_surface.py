"""CPU checks of the drop-in Python surface: names, constructor arguments,
state_dict keys and parameter-initialisation order match the reference (the
golden fixtures hold the reference's own state_dicts built under the same
seed), and the product path refuses CPU tensors instead of falling back."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import golden_io as gio
import nf.flows as nff
import nf.flows_1 as nff1
import nf.models as nfm
import nf.utils as nfu

NL = {"tanh": torch.tanh, "leaky_relu": F.leaky_relu, "elu": F.elu}


def build_layer(meta):
    kw = dict(meta["kwargs"])
    # nf/flows_1.py's own NSF_AR (flows_1.py:395-465) is a different layer
    cls = nff1.NSF_AR if meta["type"] == "NSF_AR_flows1" else getattr(nff, meta["type"])
    if meta["type"] == "Planar":
        kw["nonlinearity"] = NL[meta.get("nonlinearity", "tanh")]
    return cls(**kw)


LAYERS = [n for n in gio.names() if n.split("_")[0] in ("nsfcl", "realnvp", "planar", "radial", "nsfar",
                                                       "nsfar1", "maf", "actnorm", "onebyone")]
# fixtures whose values were set after construction (ActNorm starts at zero, flows_1.py:204-205)
_REINIT = ("mu", "log_sigma")


def _check_values(ours, sd, module):
    """Same keys; same values except re-initialised ActNorm parameters; OneByOneConv's
    P (outside the state_dict, flows_1.py:229) equals the fixture's under the same
    numpy seed."""
    keys = [k for k in sd if not (k == "P" or k.endswith(".P"))]
    assert list(ours.keys()) == keys
    for k in keys:
        if k.split(".")[-1] in _REINIT:
            continue
        torch.testing.assert_close(ours[k], sd[k], rtol=0, atol=0)
    for k in sd:
        if k == "P" or k.endswith(".P"):
            owner = module if k == "P" else module.get_submodule(k[:-2])
            torch.testing.assert_close(owner.P, sd[k], rtol=0, atol=0)


@pytest.mark.parametrize("name", LAYERS)
def test_same_seed_same_weights_and_keys(name):
    meta, _, sd = gio.load(name)
    torch.manual_seed(meta["seed"])
    np.random.seed(meta.get("np_seed", 0))
    layer = build_layer(meta)
    ours = layer.state_dict()
    if meta["type"] == "Radial":
        # the reference leaves Radial's parameters uninitialised (flows_1.py:72-83)
        assert list(ours.keys()) == list(sd.keys())
        return
    _check_values(ours, sd, layer)


@pytest.mark.parametrize("name", gio.names("model_"))
def test_model_state_dict_round_trip(name):
    meta, _, sd = gio.load(name)
    torch.manual_seed(meta["seed"])
    np.random.seed(meta["seed"])
    flows = []
    for l in meta["layers"]:
        flows.append(build_layer(dict(type=l["type"], kwargs=l["kwargs"])))
    d = meta["dim"]
    prior = torch.distributions.MultivariateNormal(torch.zeros(d), meta["var"] * torch.eye(d))
    model = nfm.NormalizingFlowModel(prior, flows)
    _check_values(model.state_dict(), sd, model)
    gio.load_into(model, sd)


def test_exports():
    for n in ("FCNN", "RealNVP", "NSF_AR", "NSF_CL", "Planar", "Radial"):
        assert hasattr(nff, n)
    import nf.flows_1 as nff1
    for n in ("FCNN", "RealNVP", "NSF_AR", "Planar", "Radial", "MAF", "ActNorm", "OneByOneConv"):
        assert hasattr(nff1, n)
    assert nfm.NormalizingFlow is nfm.NormalizingFlowModel
    assert hasattr(nfm.NormalizingFlowModel, "log_prob")
    for n in ("unconstrained_RQS", "RQS", "searchsorted", "DEFAULT_MIN_BIN_WIDTH"):
        assert hasattr(nfu, n)
    # setup.py:55-62 instantiates layers by eval() of the class name after `from nf.flows import *`
    ns = {}
    exec("from nf.flows import *", ns)
    for n in ("RealNVP", "NSF_AR", "NSF_CL"):
        assert n in ns


def test_flows_1_nsf_ar_is_its_own_layer():
    """`from nf.flows_1 import NSF_AR` binds flows_1.py:395-465: periodic
    keyword, dim nets and no init_param (nf.flows.NSF_AR has init_param and
    dim - 1 nets); its reset_parameters fails like the reference's."""
    a = nff1.NSF_AR(dim=3, K=4, B=3, hidden_dim=8)
    b = nff1.NSF_AR(dim=3, K=4, B=3, hidden_dim=8, periodic=False)
    c = nff.NSF_AR(dim=3, K=4, B=3, hidden_dim=8)
    assert len(a.layers) == 3 and not hasattr(a, "init_param")
    assert [l.network[0].in_features for l in a.layers] == [2, 2, 4]
    assert [l.network[0].in_features for l in b.layers] == [1, 1, 2]
    assert len(c.layers) == 2 and "init_param" in c.state_dict()
    with pytest.raises(AttributeError):
        a.reset_parameters()
    with pytest.raises(TypeError):
        nff.NSF_AR(dim=3, periodic=True)


def test_no_cpu_fallback():
    layer = nff.NSF_CL(size=4, dim=2, K=8, B=3, hidden_dim=8, mask=[0])
    with pytest.raises(RuntimeError, match="ROCm device only"):
        layer(torch.zeros(3, 8))
    prior = torch.distributions.MultivariateNormal(torch.zeros(8), torch.eye(8))
    model = nfm.NormalizingFlowModel(prior, [layer])
    with pytest.raises(RuntimeError, match="ROCm device only"):
        model.evaluate(torch.zeros(3, 8))
    with pytest.raises(RuntimeError, match="ROCm device only"):
        nfu.unconstrained_RQS(torch.zeros(4), torch.zeros(4, 8), torch.zeros(4, 8),
                              torch.zeros(4, 7), tail_bound=3.0)


def test_radial_and_planar_have_reference_inverse_behaviour():
    with pytest.raises(NotImplementedError):
        nff.Planar(4).inverse(torch.zeros(2, 4))
    assert not hasattr(nff.Radial(4), "inverse")


def test_nsf_cl_maps_follow_reference_layout():
    # dim=3, mask [1,2] (non-prefix): lower = coords 1,2 of each particle,
    # output puts them first in each group (flows.py:239)
    layer = nff.NSF_CL(size=2, dim=3, K=4, B=3, hidden_dim=4, mask=[1, 2])
    m = layer._maps.__func__  # no device use: call with a CPU device just to build lists
    maps = m(layer, torch.device("cpu"))
    assert maps.lo_in.tolist() == [1, 2, 4, 5]
    assert maps.up_in.tolist() == [0, 3]
    assert maps.lo_out.tolist() == [0, 1, 3, 4]
    assert maps.up_out.tolist() == [2, 5]
