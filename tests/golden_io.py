"""Load the committed golden fixtures (arrays only, no pickle)."""
import glob
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names(prefix=""):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as f:
        meta = json.loads(str(f["meta"]))
        arrays = {k: torch.from_numpy(f[k].copy()) for k in f.files if k != "meta"}
    sd = {k[3:]: v for k, v in arrays.items() if k.startswith("sd.")}
    data = {k: v for k, v in arrays.items() if not k.startswith("sd.")}
    if meta.get("sd_from_seed"):
        sd = _rebuild_sd(meta, data)
    return meta, data, sd


def _rebuild_sd(meta, data):
    """Weights of a fixture too large to hold them (make_golden.py
    case_layer_seeded): the package's layer built from the fixture's seed (the
    reference's init order), checked against the fixture's per-entry fp64 sum,
    sum of squares and first 8 values."""
    import nf.flows as nff
    torch.manual_seed(meta["seed"])
    layer = getattr(nff, meta["type"])(**meta["kwargs"])
    sd = {k: v.detach().clone() for k, v in layer.state_dict().items()}
    packed = "sd_keys" in meta
    if packed:
        assert list(sd.keys()) == meta["sd_keys"], "state_dict keys differ from the fixture's"
        all_sums, all_heads = data.pop("sdsum_all"), data.pop("sdhead_all")
    for i, (k, v) in enumerate(sd.items()):
        if packed:
            sums, head = all_sums[i], all_heads[i][:min(8, v.numel())]
        else:
            sums, head = data.pop("sdsum." + k), data.pop("sdhead." + k)
        v64 = v.double().flatten()
        got = torch.stack([v64.sum(), v64.square().sum()])
        if not (torch.equal(v.flatten()[:8], head) and torch.allclose(got, sums, rtol=1e-12, atol=1e-12)):
            raise AssertionError("%s: weights rebuilt from seed %d differ from the fixture's" % (k, meta["seed"]))
    assert not any(k.startswith(("sdsum.", "sdhead.")) for k in data), "fixture has entries the layer lacks"
    return sd


def layer_spec(meta, prefix=""):
    kw = dict(meta["kwargs"])
    spec = dict(type=meta["type"], prefix=prefix, **kw)
    if meta["type"] == "Planar":
        spec["nonlinearity"] = meta.get("nonlinearity", "tanh")
    if meta["type"] in ("NSF_CL", "NSF_AR"):
        spec.setdefault("K", 32)
        spec.setdefault("B", 3)
    if meta["type"] == "NSF_CL":
        spec.setdefault("dim", 3)
        spec.setdefault("mask", [1])
    return spec


def load_into(module, sd, strict=True):
    """load_state_dict plus OneByOneConv's permutation P, which the reference
    keeps outside the state_dict (flows_1.py:229); fixtures carry it as
    ``[<prefix>.]P``."""
    extra = {k: v for k, v in sd.items() if k == "P" or k.endswith(".P")}
    module.load_state_dict({k: v for k, v in sd.items() if k not in extra}, strict=strict)
    for k, v in extra.items():
        owner = module if k == "P" else module.get_submodule(k[:-2])
        owner.P = v.clone().to(owner.P.device)
    return module
