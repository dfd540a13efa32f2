"""CPU: the host helper (normalizingflow_amd/csrc/nfk_host.cpp) that validates
the fused NSF_AR pack of layers with thousands of parameter tensors: its key
changes exactly when the Python key (module identities, every Linear's
storage + version counter) would, and it rejects non-stock conditioners."""
import time

import pytest
import torch
from torch import nn

import nf.flows as nff


@pytest.fixture(scope="module")
def hs():
    from normalizingflow_amd import _hostbuild
    _hostbuild.build()
    from normalizingflow_amd import _nfk_host
    return _nfk_host


def _state(hs, layer):
    return hs.ar_state(layer.layers._modules, layer.init_param, nff.FCNN, nn.Linear, nn.Tanh)


def test_ar_state_tracks_every_change(hs):
    torch.manual_seed(0)
    layer = nff.NSF_AR(dim=12, K=4, B=3.0, hidden_dim=16)
    s0 = _state(hs, layer)
    assert s0 >= 0 and _state(hs, layer) == s0
    with torch.no_grad():
        layer.layers[5].network[2].bias.add_(1.0)            # in-place update: version bump
    s1 = _state(hs, layer)
    assert s1 != s0
    with torch.no_grad():
        layer.init_param.mul_(1.0)
    s2 = _state(hs, layer)
    assert s2 != s1
    layer.layers[3].network[0] = nn.Linear(8, 16)            # a replaced Linear
    s3 = _state(hs, layer)
    assert s3 != s2
    layer.layers[7].network[1] = nn.Tanh()                   # a replaced activation object
    s4 = _state(hs, layer)
    assert s4 != s3 and _state(hs, layer) == s4
    layer.layers[7].network[1] = nn.ReLU()                   # not the stock FCNN any more
    assert _state(hs, layer) == -1


def test_fingerprint_tracks_versions(hs):
    ts = [torch.zeros(3) for _ in range(5)]
    f0 = hs.fingerprint(ts)
    ts[2].add_(1)
    assert hs.fingerprint(ts) != f0
    with pytest.raises(TypeError):
        hs.fingerprint([1, 2])


def test_ar_state_fast_at_polymer_size(hs):
    """Polymer.yaml's layer (2,047 conditioners): the C++ key in a few ms (the
    Python key took ~23 ms; the walk touches ~20 K Python objects)."""
    torch.manual_seed(0)
    layer = nff.NSF_AR(dim=2048, K=32, B=0.5, hidden_dim=100)
    _state(hs, layer)
    t0 = time.perf_counter()
    for _ in range(5):
        _state(hs, layer)
    dt = (time.perf_counter() - t0) / 5
    assert dt < 15e-3, dt


def _watch(hs, layer):
    return hs.ar_watch(layer.__dict__["_parameters"], layer.__dict__["_modules"], layer.layers._modules,
                       layer.init_param, nff.FCNN, nn.Linear, nn.Tanh)


@pytest.mark.parametrize("change", ["inplace", "init_inplace", "init_replaced", "linear_replaced", "tanh_replaced",
                                    "param_replaced", "data_assigned", "cond_replaced", "cond_appended",
                                    "layers_replaced"])
def test_ar_watch_invalidated_by_every_change(hs, change):
    """The watch (dict version tags + parameter storage/version) turns invalid
    on each change that alters the pack key, and stays valid otherwise."""
    torch.manual_seed(0)
    layer = nff.NSF_AR(dim=12, K=4, B=3.0, hidden_dim=16)
    w = _watch(hs, layer)
    assert w is not None and w.valid() and w.valid()
    if change == "inplace":
        with torch.no_grad():
            layer.layers[5].network[2].bias.add_(1.0)
    elif change == "init_inplace":
        with torch.no_grad():
            layer.init_param.mul_(1.0)
    elif change == "init_replaced":
        layer.init_param = nn.Parameter(layer.init_param.detach().clone())
    elif change == "linear_replaced":
        layer.layers[3].network[0] = nn.Linear(8, 16)
    elif change == "tanh_replaced":
        layer.layers[7].network[1] = nn.Tanh()
    elif change == "param_replaced":
        layer.layers[2].network[4].weight = nn.Parameter(torch.zeros(11, 16))
    elif change == "data_assigned":
        layer.layers[4].network[0].weight.data = torch.zeros(16, 10)
    elif change == "cond_replaced":
        layer.layers[6] = nff.FCNN(14, 11, 16)
    elif change == "cond_appended":
        layer.layers.append(nff.FCNN(24, 11, 16))
    elif change == "layers_replaced":
        # a new ModuleList lives in the layer's own _modules dict, outside the
        # conditioner tree the watch walked
        layer.layers = nn.ModuleList([nff.FCNN(2 * i, 11, 16) for i in range(1, 12)])
    assert not w.valid()


def test_ar_watch_rejects_non_stock(hs):
    torch.manual_seed(0)
    layer = nff.NSF_AR(dim=6, K=4, B=3.0, hidden_dim=16)
    layer.layers[2].network[1] = nn.ReLU()
    assert _watch(hs, layer) is None


def test_ar_watch_fast_at_polymer_size(hs):
    """valid() compares the cached words only (~20 K at Polymer's 2,047
    conditioners): well under the key's recomputation."""
    torch.manual_seed(0)
    layer = nff.NSF_AR(dim=2048, K=32, B=0.5, hidden_dim=100)
    w = _watch(hs, layer)
    w.valid()
    t0 = time.perf_counter()
    for _ in range(10):
        assert w.valid()
    dt = (time.perf_counter() - t0) / 10
    assert dt < 5e-3, dt


def test_copies_and_pickles_drop_the_watch(hs):
    """A layer holding the watch a fused GPU forward leaves behind (the C++
    ArWatch in _pack_cache) deep-copies and pickles: the copy carries no derived
    state and rebuilds its own pack; the original keeps its cache."""
    import copy
    import pickle
    torch.manual_seed(0)
    layer = nff.NSF_AR(dim=6, K=4, B=3.0, hidden_dim=16)
    w = _watch(hs, layer)
    layer._pack_cache = (("cpu", ()), torch.zeros(4), 16, None, ("cpu", w))
    layer._stock_linears()
    layer._named_param_list()
    for c in (copy.deepcopy(layer), pickle.loads(pickle.dumps(layer))):
        assert c._pack_cache is None and c._ar_tree is None and c.__dict__.get("_named_cache") is None
        assert c._cols == {}
        sd, sc = layer.state_dict(), c.state_dict()
        assert sd.keys() == sc.keys() and all(torch.equal(sd[k], sc[k]) for k in sd)
        assert len(c._stock_linears()) == 3 * 5
        assert [n for n, _ in c._named_param_list()] == [n for n, _ in layer.named_parameters()]
    assert layer._pack_cache[4][1] is w and w.valid()


def test_make_watch_tracks_realnvp_tree(hs):
    """The generic watch RealNVP's weight-stream pack is cached on (module-tree
    dicts + the 24 Linear tensors): valid until a module, parameter or value changes."""
    torch.manual_seed(0)

    def watch(layer):
        nets = (layer.s1, layer.t1, layer.s2, layer.t2)
        dicts, params = [layer.__dict__["_modules"]], []
        for n in nets:
            net = n.__dict__["_modules"]["network"]
            dicts += [n.__dict__["_modules"], net.__dict__["_modules"]]
            dicts += [net.__dict__["_modules"][str(i)].__dict__["_parameters"] for i in (0, 2, 4)]
            params += [t for i in (0, 2, 4) for t in (net[i].weight, net[i].bias)]
        return hs.make_watch(dicts, params)

    for change in ("none", "inplace", "linear", "net", "param"):
        layer = nff.RealNVP(16, hidden_dim=32)
        w = watch(layer)
        if change == "inplace":
            with torch.no_grad():
                layer.s2.network[2].weight.mul_(2.0)
        elif change == "linear":
            layer.t1.network[4] = nn.Linear(32, 8)
        elif change == "net":
            layer.s1 = nff.FCNN(8, 8, 32)
        elif change == "param":
            layer.t2.network[0].bias = nn.Parameter(torch.zeros(32))
        assert w.valid() == (change == "none"), change
    with pytest.raises(TypeError):
        hs.make_watch([1], [])
