"""CPU checks of the chained NSF_CL launch (nfk_fused_nsf_chain): the composed
tile-column maps the host builds (models._compose_maps) and the host-only
parts of the C ABI (layer-count query, argument validation; no device call).

The map check is independent of the composition code: a run of NSF_CL layers
evaluated by the CPU oracle (nf/flows.py:227-253) on rows that lie entirely
outside [-B, B] is the identity per element (nf/utils.py:46-47) but still
applies the masked-first output permutation of every layer (flows.py:239), so
z[:, o] = x[:, perm[o]] reveals the column permutation the chain must end on.
"""
import pytest
import torch

import nf.flows as nff
from normalizingflow_amd import _lib
from normalizingflow_amd.models import _compose_maps, _save_maps
from oracle import nf_oracle as orc


def _run(size, dim, masks, n_layers):
    torch.manual_seed(0)
    return [nff.NSF_CL(size=size, dim=dim, K=4, B=3, hidden_dim=8, mask=masks[i % len(masks)])
            for i in range(n_layers)]


@pytest.mark.parametrize("size,dim,masks,n", [
    (4, 2, [[0], [1]], 5),        # c3's alternating masks
    (3, 3, [[1], [0, 2], [2]], 4),  # dim 3, non-prefix and two-coordinate masks
    (5, 2, [[1]], 3),              # the same non-prefix mask every layer
])
def test_composed_maps_match_oracle_permutation(size, dim, masks, n):
    run = _run(size, dim, masks, n)
    D = size * dim
    cm = _compose_maps(run, D, torch.device("cpu")).tolist()
    assert len(cm) == n * D + D
    perm = cm[n * D:]
    assert sorted(perm) == list(range(D))
    # rows 1.. entirely outside the spline interval: identity values, permuted columns
    x = torch.empty(3, D)
    x[0] = 0.1                                  # one inside row (the oracle needs one)
    x[1:] = 10.0 + torch.arange(D, dtype=torch.float32)
    specs = [dict(type="NSF_CL", prefix="%d." % i, size=size, dim=dim, K=4, B=3, mask=list(f.mask.tolist()))
             for i, f in enumerate(run)]
    sd = {"%d.%s" % (i, k): v for i, f in enumerate(run) for k, v in f.state_dict().items()}
    z = x
    for s in specs:
        z, _ = orc.apply_layer(s, z, sd)
    assert [int(v) - 10 for v in z[1].tolist()] == perm
    # every layer's lower/upper tile columns: the layer's inputs under the
    # permutation of the layers before it
    p = list(range(D))
    for i, f in enumerate(run):
        lo_in, lo_out, up_in, up_out = f._maps(torch.device("cpu")).lists
        assert cm[i * D:i * D + len(lo_in)] == [p[c] for c in lo_in]
        assert cm[i * D + len(lo_in):(i + 1) * D] == [p[c] for c in up_in]
        q = [0] * D
        for o, c in list(zip(lo_out, lo_in)) + list(zip(up_out, up_in)):
            q[o] = p[c]
        p = q


@pytest.mark.parametrize("size,dim,masks,n", [
    (4, 2, [[0], [1]], 5),
    (3, 3, [[1], [0, 2], [2]], 4),
])
def test_save_maps_are_the_layer_inputs(size, dim, masks, n):
    """nfk_fused_nsf_chain_saved's smaps (models._save_maps): for layer l >= 1,
    column j of that layer's input sits in the tile column the chain's cmaps
    give for it (its lower / upper input lists), and the permutation after the
    last layer is cmaps' output map."""
    run = _run(size, dim, masks, n)
    D = size * dim
    cm = _compose_maps(run, D, torch.device("cpu")).tolist()
    sm = _save_maps(run, D, torch.device("cpu")).tolist()
    assert len(sm) == (n - 1) * D
    for i in range(1, n):
        lo_in, _, up_in, _ = run[i]._maps(torch.device("cpu")).lists
        smi = sm[(i - 1) * D:i * D]
        assert sorted(smi) == list(range(D))
        assert [smi[c] for c in lo_in] == cm[i * D:i * D + len(lo_in)]
        assert [smi[c] for c in up_in] == cm[i * D + len(lo_in):(i + 1) * D]


def test_chain_saved_validation_is_host_only():
    lib = _lib.load()
    assert lib.nfk_fused_nsf_chain_saved_ok(32, 32, 100, 8, 8) == 1     # c3: the two-tile chain
    assert lib.nfk_fused_nsf_chain_saved_ok(32, 32, 100, 8, 1) == 0     # one layer: no chain
    assert lib.nfk_fused_nsf_chain_saved_ok(32, 32, 64, 8, 8) == 0      # not a two-tile-chain shape
    args = lambda nl, x=16, sv=16, st=256 * 64: (x, 64, 16, 16, nl, 32, 32, 100, 16, 64, 16, 1, 256, 8, 3.0,
                                                  None, sv, 64, st, 16, None)
    assert lib.nfk_fused_nsf_chain_saved(*args(1)) == _lib.NFK_EINVAL
    assert b"layer count" in lib.nfk_last_error()
    assert lib.nfk_fused_nsf_chain_saved(*args(8, sv=None)) == _lib.NFK_EINVAL
    assert b"null pointer" in lib.nfk_last_error()
    assert lib.nfk_fused_nsf_chain_saved(*args(8, x=4)) == _lib.NFK_EINVAL
    assert b"aligned" in lib.nfk_last_error()
    assert lib.nfk_fused_nsf_chain_saved(*args(8, st=64)) == _lib.NFK_EINVAL   # layer stride < batch rows


def test_chain_layer_count_query_is_host_only():
    lib = _lib.load()
    n = lib.nfk_fused_nsf_chain_max(32, 32, 100, 8)   # c3 layer shape
    assert n >= 8                                      # the c3 model runs as one launch
    assert lib.nfk_fused_nsf_chain_max(32, 32, 256, 8) == 0   # no narrow kernel for H = 256
    assert lib.nfk_fused_nsf_chain_max(33, 32, 100, 8) == 0   # D % 4 != 0: no split form


def test_chain_argument_validation_is_host_only():
    lib = _lib.load()
    nmax = lib.nfk_fused_nsf_chain_max(32, 32, 100, 8)
    args = lambda nl, x=16, z=16, lp=None, sc=1.0: (x, 64, 16, 16, nl, 32, 32, 100, z, 64, None, 0, 256, 8,
                                                    3.0, 0, None, lp, sc, 0.0, None)
    assert lib.nfk_fused_nsf_chain(*args(0)) == _lib.NFK_EINVAL
    assert b"layer count" in lib.nfk_last_error()
    assert lib.nfk_fused_nsf_chain(*args(nmax + 1)) == _lib.NFK_EINVAL
    assert lib.nfk_fused_nsf_chain(*args(2, x=4)) == _lib.NFK_EINVAL
    assert b"aligned" in lib.nfk_last_error()
    rc = lib.nfk_fused_nsf_chain(16, 64, 16, 16, 2, 32, 32, 100, 16, 64, None, 1, 256, 8, 3.0, 0, None,
                                 None, 1.0, 0.0, None)
    assert rc == _lib.NFK_EINVAL and b"null logdet" in lib.nfk_last_error()
    assert lib.nfk_fused_nsf_chain(*args(2, z=None)) == _lib.NFK_EINVAL      # neither z nor log_prob
    assert b"null pointer" in lib.nfk_last_error()
    assert lib.nfk_fused_nsf_chain(*args(2, z=None, lp=16, sc=0.0)) == _lib.NFK_EINVAL
    assert b"prior scale" in lib.nfk_last_error()


def test_layer_grouping(monkeypatch):
    """NormalizingFlowModel._groups: runs of consecutive same-shape fused NSF_CL
    layers become (run, shape) items of at most nfk_fused_nsf_chain_max layers;
    other layers, shape changes and single-layer runs stay per-layer; training
    (grad) chains only NSF_CL runs in the forward direction that the
    saved-input chain takes.  Fused-kernel availability is stubbed (no device)."""
    import nf.models as nfm
    from normalizingflow_amd import config
    from normalizingflow_amd import kernels as K_
    torch.manual_seed(0)
    a = [nff.NSF_CL(size=4, dim=2, K=4, B=3, hidden_dim=8, mask=[i % 2]) for i in range(5)]
    b = nff.NSF_CL(size=4, dim=2, K=6, B=3, hidden_dim=8, mask=[0])     # another K
    r = nff.RealNVP(8, hidden_dim=8)
    monkeypatch.setattr(nff.NSF_CL, "_chain_shape",
                        lambda self, dev: (4, 4, 8, self.K, float(self.B)))
    monkeypatch.setattr(K_, "fused_nsf_chain_max", lambda *s: 3)
    monkeypatch.setattr(config, "USE_FUSED", True)
    monkeypatch.setattr(config, "USE_CHAIN", True)
    flows = [a[0], a[1], r, a[2], a[3], a[4], b, a[0]]
    m = nfm.NormalizingFlowModel(None, flows)
    g = m._groups(m.flows, torch.device("cpu"), False)
    kinds = [("run", [flows.index(f) for f in it[0]]) if isinstance(it, tuple) else ("one", flows.index(it))
             for it in g]
    assert kinds == [("run", [0, 1]), ("one", 2), ("run", [3, 4, 5]), ("one", 6), ("one", 0)]
    assert g[0][1] == (4, 4, 8, 4, 3.0)
    # longer than one launch: 5 same-shape layers with capacity 3 -> 3 + 2
    m2 = nfm.NormalizingFlowModel(None, a)
    g2 = m2._groups(m2.flows, torch.device("cpu"), False)
    assert [len(it[0]) for it in g2] == [3, 2]
    # capacity 1 (or 0): no chains at all
    monkeypatch.setattr(K_, "fused_nsf_chain_max", lambda *s: 0)
    assert m2._groups(m2.flows, torch.device("cpu"), False) == list(a)
    assert m._groups(m.flows, torch.device("cpu"), True) == flows
    # training (grad): NSF_CL runs the saved-input chain takes, forward only
    monkeypatch.setattr(K_, "fused_nsf_chain_max", lambda *s: 3)
    monkeypatch.setattr(K_, "fused_nsf_chain_saved_ok", lambda *s: True)
    g3 = m._groups(m.flows, torch.device("cpu"), True)
    kinds3 = [("run", [flows.index(f) for f in it[0]]) if isinstance(it, tuple) else ("one", flows.index(it))
              for it in g3]
    assert kinds3 == [("run", [0, 1]), ("one", 2), ("run", [3, 4, 5]), ("one", 6), ("one", 0)]
    assert m._groups(m.flows, torch.device("cpu"), True, inverse=True) == flows
    monkeypatch.setattr(K_, "fused_nsf_chain_saved_ok", lambda *s: False)
    assert m._groups(m.flows, torch.device("cpu"), True) == flows
    monkeypatch.setattr(K_, "fused_nsf_chain_saved_ok", lambda *s: True)
    monkeypatch.setattr(config, "USE_TRAIN_CHAIN", False)
    assert m._groups(m.flows, torch.device("cpu"), True) == flows
    # RealNVP runs are not grouped under grad
    rr = [nff.RealNVP(8, hidden_dim=8) for _ in range(3)]
    monkeypatch.setattr(config, "USE_TRAIN_CHAIN", True)
    monkeypatch.setattr(nff.RealNVP, "_chain_shape", lambda self, dev: ("rnvp", 16, 8, 4))
    monkeypatch.setattr(K_, "fused_realnvp_chain_max", lambda *s: 8)
    mr = nfm.NormalizingFlowModel(None, rr)
    assert isinstance(mr._groups(mr.flows, torch.device("cpu"), False)[0], tuple)
    assert mr._groups(mr.flows, torch.device("cpu"), True) == rr
    monkeypatch.setattr(config, "USE_CHAIN", False)
    assert m._groups(m.flows, torch.device("cpu"), False) == flows
