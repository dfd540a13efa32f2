"""Experiment configs and checkpoints of the reference's applications layer,
restated for the flow path.

* ``get_cfg_defaults`` / ``read_input`` -- the yacs defaults of
  applications/src/config.py:3-69 and the YAML merge of setup.py:84-88, with a
  small attribute-dict node (yacs is not a dependency here).  As with yacs,
  merging a key the defaults do not define raises ``KeyError``.
* ``build_flows`` / ``build_model`` -- the flow construction of
  setup.py:37-63 (RealNVP / NSF_AR / NSF_CL with the reference's tail bound B
  and NSF_CL mask cycle), the "Normal" prior of setup.py:25-30.  Other
  potentials/priors (LJ, Fe, Einstein crystal, Gaussian mixtures) belong to
  the physics layer and are out of scope.
* ``save_checkpoint`` / ``load_checkpoint`` -- the checkpoint dict of
  train.py:39-40 and the loader of setup.py:102-109 (``load_state_dict``
  with ``strict=False``), read with ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import ast
import copy

import torch
import yaml

from . import flows as F_
from .models import NormalizingFlowModel

__all__ = ["CfgNode", "get_cfg_defaults", "read_input", "tail_bound", "build_flows", "build_prior",
           "build_model", "save_checkpoint", "load_checkpoint", "train_step"]


class CfgNode(dict):
    """Nested attribute dictionary with yacs-style ``merge_from_file``."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def clone(self):
        return copy.deepcopy(self)

    def merge_from_dict(self, d, path=""):
        for k, v in d.items():
            if k not in self:
                raise KeyError("Non-existent config key: %s%s" % (path, k))
            if isinstance(self[k], CfgNode):
                if not isinstance(v, dict):
                    raise ValueError("config key %s%s must be a mapping" % (path, k))
                self[k].merge_from_dict(v, path + k + ".")
            else:
                self[k] = _decode(v)

    def merge_from_file(self, filename):
        with open(filename) as f:
            self.merge_from_dict(yaml.safe_load(f) or {})


def _decode(v):
    """yacs decodes string values with ast.literal_eval ("5e-3" -> 0.005; YAML
    itself reads an exponent without a dot as a string)."""
    if isinstance(v, str):
        try:
            return ast.literal_eval(v)
        except (ValueError, SyntaxError):
            return v
    return v


def _node(**kw):
    n = CfgNode()
    for k, v in kw.items():
        n[k] = v
    return n


def get_cfg_defaults():
    """applications/src/config.py:3-69."""
    dataset = _node(name=None, potential=None, training_data=None, testing_data=None, data=None,
                    nparticles=32, dim=3, kT=1.0, rho=None, ncellx=None, ncelly=None, ncellz=None,
                    cell_len=None, boxlength=None, periodic=True, type="xyz", sigma=1.0,
                    epsilon=1.0, cutoff=1.6, shift=True, centers=None, vars=None, alpha=None,
                    input_dir=None)
    return _node(
        device="cuda:0",
        dataset=dataset,
        flow=_node(type="NSF_AR", nlayers=3, nsplines=32, hidden_dim=100),
        # prior.nparticles/dim/boxlength are copies of the dataset defaults (config.py:48-50)
        prior=_node(type=None, lattice_dir=None, alpha=100, centers=None, vars=None,
                    nparticles=32, dim=3, boxlength=None),
        train_parameters=_node(max_epochs=4000, batch_size=100, output_freq=100,
                               learning_rate=1e-4, scheduler="exponential",
                               lr_scheduler_gamma=0.999),
        output=_node(training_dir="../training/", testing_dir="../testing/",
                     model_dir="../saved_models/", best_model_dir="../trained_models/"))


def read_input(path):
    """setup.py:84-88 (without the print)."""
    cfg = get_cfg_defaults()
    cfg.merge_from_file(path)
    return cfg


def tail_bound(cfg):
    """The spline tail bound B of setup.py:38-44 (None when the config sets
    neither rho nor ncellx; the reference then fails only if it needs B)."""
    d = cfg.dataset
    if d.rho is not None:
        return (d.nparticles / (8 * d.rho)) ** (1 / 3)
    if d.ncellx is not None:
        return d.ncellx * d.cell_len / 2
    return None


def build_flows(cfg):
    """setup.py:55-62."""
    N = cfg.dataset.nparticles * cfg.dataset.dim
    fl = cfg.flow
    B = tail_bound(cfg)
    if fl.type == "RealNVP":
        return [F_.RealNVP(dim=N, hidden_dim=fl.hidden_dim) for _ in range(fl.nlayers)]
    if B is None:
        raise NameError("name 'B' is not defined (set dataset.rho or dataset.ncellx)")
    if fl.type == "NSF_AR":
        return [F_.NSF_AR(dim=N, K=fl.nsplines, B=B, hidden_dim=fl.hidden_dim, device=cfg.device)
                for _ in range(fl.nlayers)]
    if fl.type == "NSF_CL":
        cycle = [[0], [1], [2], [0, 1], [1, 2], [0, 2]]
        masks = sum([cycle for _ in range(fl.nlayers // 6 + 1)], [])[:fl.nlayers]
        return [F_.NSF_CL(size=cfg.dataset.nparticles, dim=3, K=fl.nsplines, B=B,
                          hidden_dim=fl.hidden_dim, mask=masks[i], device=cfg.device)
                for i in range(fl.nlayers)]
    raise ValueError("flow type %r is not built by setup.py" % fl.type)


def build_prior(cfg, device):
    """The "Normal" prior of setup.py:25-30."""
    p = cfg.prior
    if p.type != "Normal":
        raise NotImplementedError("prior %r lives in the physics layer (out of scope); pass a "
                                  "prior object to build_model" % p.type)
    N = p.nparticles * p.dim
    var = 1 if p.vars is None else p.vars
    return torch.distributions.MultivariateNormal(torch.zeros(N, device=device),
                                                  var * torch.eye(N, device=device))


def build_model(cfg, prior=None, device=None):
    """NormalizingFlowModel(prior, flows, cfg.device).to(device) (setup.py:63)."""
    device = cfg.device if device is None else device
    prior = build_prior(cfg, device) if prior is None else prior
    if cfg.dataset.boxlength is None and tail_bound(cfg) is not None:
        cfg.dataset.boxlength = 2 * tail_bound(cfg)
    return NormalizingFlowModel(prior, build_flows(cfg), device).to(device)


def save_checkpoint(path, model, optimizer=None, scheduler=None, epoch=0, losses=()):
    """train.py:39-40: {"model", "optim", "scheduler", "epoch", "loss"}."""
    torch.save({"model": model.state_dict(),
                "optim": None if optimizer is None else optimizer.state_dict(),
                "scheduler": None if scheduler is None else scheduler.state_dict(),
                "epoch": epoch,
                "loss": [float(v) for v in losses]}, path)


def load_checkpoint(model, path, optimizer=None, scheduler=None):
    """setup.py:102-109: load the "model" entry with strict=False (weights only;
    nothing in the file is executed).  Returns the checkpoint dict."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(ck["model"], strict=False)
    if optimizer is not None and ck.get("optim") is not None:
        optimizer.load_state_dict(ck["optim"])
    if scheduler is not None and ck.get("scheduler") is not None:
        scheduler.load_state_dict(ck["scheduler"])
    return ck


def train_step(model, optimizer, x, scheduler=None):
    """One iteration of train.py:21-29: forward KL / NLL, backward, step."""
    optimizer.zero_grad()
    z, prior_logprob, log_det = model(x)
    loss = -torch.mean(prior_logprob + log_det)
    loss.backward()
    optimizer.step()
    if scheduler is not None:
        scheduler.step()
    return loss.detach()
