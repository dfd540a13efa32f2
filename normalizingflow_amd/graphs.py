"""log_prob / sample of a fixed batch shape as one HIP graph.

A small batch (BASELINE c1: 4096 rows of a 4-layer RealNVP with D = 2, whose
conditioners are library GEMMs) is launch-bound: ~90 kernel launches per
log_prob, each a few microseconds of host work.  ``GraphedLogProb`` captures
one ``model.log_prob`` call on a static input buffer into a HIP graph
(``torch.cuda.CUDAGraph``, hipGraph on ROCm) and replays it: one launch per
call, the same kernels and the same results (bitwise: the replay runs the
captured kernels on the same buffers).

The reference has no counterpart (nf/models.py:37-40 is eager PyTorch); the
call signature and results are those of ``NormalizingFlowModel.log_prob``.

Contract:
  * the batch shape, dtype and device are fixed at capture; ``__call__(x)``
    copies x into the static input (or pass None after writing ``.x``);
  * the returned tensor is the graph's static output, overwritten by the
    next replay (clone it to keep it);
  * the weights are baked in as the packed buffers of the capture: the graph
    holds strong references to every cache entry the captured call used (the
    layers' weight packs, the chained-launch pointer tables and maps, the
    log_prob plan), so an eager call or ``invalidate_caches()`` after a
    parameter update cannot free memory the graph reads; ``replay()`` compares
    the parameters' (storage, version) with those of the capture and
    recaptures when they changed (``recapture()`` does it by hand, e.g. after
    writes through ``p.data`` that bump no version);
  * the reference's errors (status words of the spline layers and the prior)
    are checked after every replay per ``config.STRICT_CHECKS``, like an
    eager call ("deferred": raised by a later call or flush_status_checks()).
"""
from __future__ import annotations

import torch

from . import flows as _flows
from .flows import check_status, flush_status_checks


_CACHE_ATTRS = ("_pack_cache", "_vjp_cache", "_chain_cache", "_lp_plan_cache")


def _cache_refs(model):
    """Strong references to every parameter-derived cache entry of ``model``
    (the buffers a captured call's kernels read by raw pointer)."""
    refs = []
    for m in model.modules():
        for name in _CACHE_ATTRS:
            v = m.__dict__.get(name)
            if v is None:
                continue
            refs.append(tuple(v.values()) if isinstance(v, dict) else v)
    return refs


def _param_key(model):
    return tuple((p.data_ptr(), p._version) for p in model.parameters())


def _param_watch(model):
    """A C++ watch (nfk_host.cpp make_watch) over every module's parameter and
    submodule dicts (CPython version tags: a replaced module or parameter) and
    every parameter's (storage, offset, version): the staleness test of
    ``_param_key`` in microseconds -- the key walked all 12,288 parameters of a
    Polymer NSF_AR model per replay, ~30 ms.  None without the helper."""
    hs = _flows._host_helper()
    if hs is None:
        return None
    dicts = []
    for m in model.modules():
        dicts.append(m.__dict__["_parameters"])
        dicts.append(m.__dict__["_modules"])
    return hs.make_watch(dicts, list(model.parameters()))


class _Graphed:
    """A no-argument call ``fn`` on ``device`` captured once and replayed.
    With ``model`` the capture pins the model's caches and replays recapture
    when its parameters changed."""

    def __init__(self, fn, device, warmup=2, model=None):
        if torch.device(device).type != "cuda":
            raise ValueError("graph capture needs a HIP device (got %s)" % device)
        self._fn = fn
        self._device = torch.device(device)
        self._warmup = warmup
        self._model = model
        self._keep = []
        self._key = None
        self._watch = None
        self.graph = None
        self.out = None
        self._status = []
        self.recapture()

    def recapture(self):
        """(Re)capture the call: eager warm-up calls on a side stream fill the
        model's weight-pack and plan caches (no allocation or host copy may
        happen under capture), then one call is captured."""
        dev = self._device
        side = torch.cuda.Stream(dev)
        cur = torch.cuda.current_stream(dev)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(self._warmup):
                self._fn()
        cur.wait_stream(side)
        torch.cuda.synchronize(dev)
        flush_status_checks()  # the warm-up's errors surface here, before capture
        self.graph = torch.cuda.CUDAGraph()
        sink = []
        prev, _flows._CAPTURE_SINK = _flows._CAPTURE_SINK, sink
        try:
            with torch.cuda.graph(self.graph):
                self.out = self._fn()
        finally:
            _flows._CAPTURE_SINK = prev
        self._status = sink
        if self._model is not None:
            # the capture's packs, pointer tables and plan live as long as the graph
            self._keep = _cache_refs(self._model)
            self._key = _param_key(self._model)
            self._watch = _param_watch(self._model)
        return self

    def stale(self):
        """True when the model's parameters changed since the capture."""
        if self._model is None:
            return False
        if self._watch is not None:
            return not self._watch.valid()
        return _param_key(self._model) != self._key

    def replay(self):
        if self.stale():
            self.recapture()
        self.graph.replay()
        for status, n, prior in self._status:
            check_status(status, n, prior)
        return self.out


class GraphedLogProb(_Graphed):
    """``model.log_prob`` on batches of ``example_x``'s shape as one graph replay."""

    def __init__(self, model, example_x, warmup=2):
        self.x = example_x.detach().clone()
        super().__init__(lambda: model.log_prob(self.x), self.x.device, warmup, model=model)

    def __call__(self, x=None):
        if x is not None:
            if x.shape != self.x.shape or x.dtype != self.x.dtype:
                raise ValueError("graphed call captured for %s %s, got %s %s"
                                 % (tuple(self.x.shape), self.x.dtype, tuple(x.shape), x.dtype))
            self.x.copy_(x)
        return self.replay()


class GraphedSample(_Graphed):
    """``model.sample(n)`` as one graph replay: the prior draw (torch's device
    generator, graph-safe: every replay draws fresh values), the inverse chain
    and the prior log-density.  Returns the graph's static (x, log_px, z)."""

    def __init__(self, model, n_samples, warmup=2):
        self.n = int(n_samples)
        super().__init__(lambda: model.sample(self.n), model.prior.loc.device, warmup, model=model)

    def __call__(self):
        return self.replay()
