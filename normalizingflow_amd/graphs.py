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
  * the weights are baked in as the packed buffers of the capture: after a
    parameter update call ``recapture()`` (the model's caches are keyed on
    parameter versions, so eager calls are never stale, but a graph is);
  * the reference's errors (status words of the spline layers and the prior)
    are checked after every replay per ``config.STRICT_CHECKS``, like an
    eager call ("deferred": raised by a later call or flush_status_checks()).
"""
from __future__ import annotations

import torch

from . import flows as _flows
from .flows import check_status, flush_status_checks


class _Graphed:
    """A no-argument call ``fn`` on ``device`` captured once and replayed."""

    def __init__(self, fn, device, warmup=2):
        if torch.device(device).type != "cuda":
            raise ValueError("graph capture needs a HIP device (got %s)" % device)
        self._fn = fn
        self._device = torch.device(device)
        self._warmup = warmup
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
        return self

    def replay(self):
        self.graph.replay()
        for status, n, prior in self._status:
            check_status(status, n, prior)
        return self.out


class GraphedLogProb(_Graphed):
    """``model.log_prob`` on batches of ``example_x``'s shape as one graph replay."""

    def __init__(self, model, example_x, warmup=2):
        self.x = example_x.detach().clone()
        super().__init__(lambda: model.log_prob(self.x), self.x.device, warmup)

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
        super().__init__(lambda: model.sample(self.n), model.prior.loc.device, warmup)

    def __call__(self):
        return self.replay()
