"""Flow layers with the reference's class surface, backed by HIP kernels.

Drop-in for ``nf.flows`` / ``nf.flows_1`` of sherryli59/NormalizingFlow: same
class names, constructor arguments, attributes, ``forward``/``inverse``
signatures, return shapes, parameter-initialisation order (so a given
``torch.manual_seed`` yields the same weights) and ``state_dict`` keys.

What runs where (ROCm device only -- CPU tensors raise, there is no fallback):
  FCNN           stock nn.Linear/Tanh stack (library GEMMs) -- flows.py:20-35
  NSF_CL         fused MFMA conditioner + spline kernel (nfk_fused_nsf) when the
                 shape is supported, else FCNN + nfk_rqs_coupling -- flows.py:210-253
  RealNVP        4 FCNN + nfk_affine_coupling per half -- flows.py:38-76
  NSF_AR         per-dimension FCNN on nfk_trig_features + nfk_rqs_coupling
                 -- flows.py:152-209
  Planar         nfk_planar -- flows_1.py:21-63
  Radial         nfk_radial_sumsq (+ optional all-reduce) + nfk_radial_apply
                 -- flows_1.py:66-97
  MAF            per-coordinate FCNN conditioners + nfk_maf -- flows_1.py:159-195
  ActNorm        nfk_actnorm -- flows_1.py:198-215
  OneByOneConv   x @ P @ L @ (U + diag S) as library GEMMs -- flows_1.py:218-252
Gradients: when autograd needs them (grad mode on and x or a parameter
requires grad) a layer runs as ``_LayerFn``: the forward is the same HIP
kernel chain; backward starts from the saved input (activation memory = one
input per layer, like gradient checkpointing) and runs hand-written kernels:
nfk_fused_nsf_vjp (NSF_CL conditioner recompute + spline VJP), fcnn_grad
(conditioner backward), nfk_affine_coupling_bwd (RealNVP) and the per-row
VJP kernels of nfk_flows_bwd.hip (Planar, Radial, ActNorm, MAF, NSF_AR).
Only user-supplied (non-FCNN) conditioners back-propagate through the
differentiable torch restatement (``torch_math``).
"""
from __future__ import annotations

import collections
import functools

import math
import warnings

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.nn.init as init

from . import config
from . import fcnn_grad
from . import kernels as K_
from . import torch_math
from ._lib import ST_INSIDE_SEEN, ST_NAN_Z, ST_NEG_DISC

__all__ = ["FCNN", "RealNVP", "NSF_AR", "NSF_CL", "Planar", "Radial", "MAF", "ActNorm",
           "OneByOneConv", "functional_derivatives"]

# flows.py:12-18 -- kept for API parity (used by Planar's CPU reference semantics)
functional_derivatives = {
    torch.tanh: lambda x: 1 - torch.pow(torch.tanh(x), 2),
    F.leaky_relu: lambda x: (x > 0).type(x.dtype) + (x < 0).type(x.dtype) * -0.01,
    F.elu: lambda x: (x > 0).type(x.dtype) + (x < 0).type(x.dtype) * torch.exp(x),
}

def _needs_grad(module, x):
    return torch.is_grad_enabled() and (
        x.requires_grad or any(p.requires_grad for p in module.parameters()))


class _LayerFn(torch.autograd.Function):
    """One layer as an autograd node: HIP forward, recompute-backward.

    forward(layer, inverse, status, names, x, *params) -> (z, logdet)
    backward recomputes (z, logdet) = torch_math.layer_forward(...) from the
    saved x and parameters under enable_grad and returns their vector-Jacobian
    products.  The kernels' outputs are the values the graph continues from;
    the recomputation only supplies derivatives.
    """

    @staticmethod
    def forward(ctx, layer, inverse, status, names, x, *params):
        ctx.layer, ctx.inverse, ctx.names = layer, inverse, names
        ctx.save_for_backward(x, *params)
        return layer._eval(x, inverse, status)

    @staticmethod
    def backward(ctx, gz, gld):
        x, *params = ctx.saved_tensors
        need = ctx.needs_input_grad[4:]
        vjp = getattr(ctx.layer, "_vjp", None)
        if vjp is not None:
            return (None, None, None, None, *vjp(x, ctx.names, params, gz, gld, ctx.inverse, need))
        with torch.enable_grad():
            xd = x.detach().requires_grad_(need[0])
            pd = [p.detach().requires_grad_(n) for p, n in zip(params, need[1:])]
            z, ld = torch_math.layer_forward(ctx.layer, xd, dict(zip(ctx.names, pd)), ctx.inverse)
            outs, grads_out = [], []
            for o, g in ((z, gz), (ld, gld)):
                if g is not None and o.requires_grad:
                    outs.append(o)
                    grads_out.append(g.expand_as(o) if g.shape != o.shape else g)
            inputs = [t for t in [xd] + pd if t.requires_grad]
            got = (torch.autograd.grad(outs, inputs, grads_out, allow_unused=True)
                   if outs and inputs else [None] * len(inputs))
        it = iter(got)
        res = [next(it) if t.requires_grad else None for t in [xd] + pd]
        return (None, None, None, None, *res)


def _check_input(x, what="x"):
    if not torch.is_tensor(x) or x.dim() != 2:
        raise ValueError("%s must be a 2-D tensor [batch, features]" % what)
    if not x.is_cuda:
        raise RuntimeError(
            "normalizingflow_amd runs on the ROCm device only (got a %s tensor); move the model "
            "and data to 'cuda' -- there is no CPU fallback" % x.device)
    if x.dtype != torch.float32:
        raise TypeError("normalizingflow_amd kernels compute in float32; got %s" % x.dtype)
    return x


def _validates(prior):
    """True when ``prior`` validates its arguments (torch's support check)."""
    return prior is not None and bool(getattr(prior, "_validate_args", False))


def raise_on_status(status, n_slots=None, prior=None):
    """Reference-compatible errors from the kernels' status words (one sync).

    Slots [0, n_slots) are the spline layers' words in execution order; each
    raises what its reference layer would, in the reference's order: no
    element inside the tails first (torch.min of an empty tensor in RQS,
    utils.py:63), then a negative discriminant (utils.py:121).  NFK_ST_NAN_Z
    in any word (a NaN in z reached the Normal prior) raises torch's
    ValueError when ``prior`` validates its arguments (MultivariateNormal's
    support check in prior.log_prob, models.py:19), after every layer."""
    if status is None or (n_slots == 0 and not _validates(prior)):
        return  # nothing this word set can raise: no device->host read
    st = status.cpu().numpy()
    n = len(st) if n_slots is None else n_slots
    # the first word (in execution order) that raises decides which error
    bad = np.flatnonzero(((st[:n] & ST_INSIDE_SEEN) == 0) | ((st[:n] & ST_NEG_DISC) != 0))
    if bad.size:
        if not st[bad[0]] & ST_INSIDE_SEEN:
            raise RuntimeError("min(): Expected reduction dim to be specified for input.numel() == 0. "
                               "(no element inside the spline interval [-B, B], nf/utils.py:63)")
        raise AssertionError("negative discriminant in the inverse rational-quadratic spline "
                             "(nf/utils.py:121)")
    if _validates(prior) and bool((st & ST_NAN_Z).any()):
        raise ValueError("Expected value argument to be within the support (IndependentConstraint("
                         "Real(), 1)) of the distribution %s, but found invalid values (NaN in z)"
                         % type(prior).__name__)


class _StatusQueue:
    """config.STRICT_CHECKS == "deferred": a call's status words are copied to
    pinned host memory without a sync (a copy and an event on the call's
    stream); the errors they hold are raised at the start of a later checked
    call once the copy has landed, or by flush_status_checks().  The GPU queue
    is never drained for a check, so back-to-back calls keep the device busy."""

    MAX_PENDING = 64

    def __init__(self):
        self.pending = collections.deque()
        self.free = {}

    def _host(self, n):
        lst = self.free.get(n)
        return lst.pop() if lst else torch.empty(n, dtype=torch.int32, pin_memory=True)

    def push(self, status, n_slots, prior):
        h = self._host(status.numel())
        h.copy_(status, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(status.device))
        self.pending.append((ev, h, n_slots, prior))
        if len(self.pending) > self.MAX_PENDING:
            self.poll(block=True, upto=len(self.pending) - self.MAX_PENDING)

    def poll(self, block=False, upto=None):
        done = 0
        while self.pending and (upto is None or done < upto):
            ev, h, n, prior = self.pending[0]
            if not block and not ev.query():
                break
            ev.synchronize()
            self.pending.popleft()
            done += 1
            vals = h.clone()
            self.free.setdefault(h.numel(), []).append(h)
            raise_on_status(vals, n, prior)


_STATUS_QUEUE = _StatusQueue()


# graphs.GraphedLogProb: while a call is being captured into a HIP graph its
# status words are collected here (no host read can be captured) and checked
# after each replay instead
_CAPTURE_SINK = None


def check_status(status, n_slots=None, prior=None):
    """Raise the reference's errors for ``status`` per config.STRICT_CHECKS:
    True -> now (one device->host read, which waits for the kernels);
    "deferred" -> at a later call or flush_status_checks(); False -> never."""
    if _CAPTURE_SINK is not None and status is not None:
        _CAPTURE_SINK.append((status, n_slots, prior))
        return
    mode = config.STRICT_CHECKS
    if not mode or status is None or (n_slots == 0 and not _validates(prior)):
        return
    if mode == "deferred":
        # an earlier call's error raised by the poll must not drop this call's
        # words: they are queued either way (and checked by a later call)
        try:
            _STATUS_QUEUE.poll()
        finally:
            _STATUS_QUEUE.push(status, n_slots, prior)
    else:
        raise_on_status(status, n_slots, prior)


def flush_status_checks():
    """Wait for every deferred status check and raise the first error found."""
    _STATUS_QUEUE.poll(block=True)


def _invalidate_after_load(module, _incompatible_keys):
    """load_state_dict post-hook (a module-level function, so modules still pickle)."""
    module.invalidate_caches()


class _HipFlow(nn.Module):
    """Base of the kernel-backed layers.

    ``_run(x, inverse, logdet, mode, status)`` enqueues the layer and returns z;
    ``logdet`` is written (mode 1) or accumulated (mode 2) in place, so a model
    chains layers without temporaries or syncs.  ``_n_status`` status words
    are needed per call (spline layers only).
    """
    _n_status = 0

    def __init__(self):
        super().__init__()
        # load_state_dict copies in place (a version bump the caches see), but
        # assign=True swaps tensors: drop the derived state either way
        self.register_load_state_dict_post_hook(_invalidate_after_load)

    def invalidate_caches(self):
        """Drop state derived from the parameters (fused weight packs, cached
        inverses).  The caches are keyed on each parameter's storage and
        version counter, which every autograd-visible in-place update
        (optimizer steps, ``with torch.no_grad(): p.add_(...)``,
        ``load_state_dict``) bumps.  Writes through ``p.data`` do not bump it:
        call this (or NormalizingFlowModel.invalidate_caches) after them."""
        for name in ("_pack_cache", "_winv_key", "_vjp_cache", "_wide_cache"):
            if name in self.__dict__:
                self.__dict__[name] = None

    def __getstate__(self):
        """Copies and pickles (copy.deepcopy, torch.save of the module) carry no
        derived state: the packs are device buffers keyed on this object's
        parameters, the fingerprints hold object ids, and NSF_AR's pack watch is
        a C++ object (csrc/nfk_host.cpp) that neither copies nor pickles."""
        state = super().__getstate__()
        for name in _DERIVED_STATE:
            if name in state:
                state[name] = None
        if "_cols" in state:
            state["_cols"] = {}
        return state

    def _named_param_list(self):
        """[(name, parameter)] for the autograd node (named_parameters order)."""
        return list(self.named_parameters())

    def _run(self, x, inverse, logdet, mode, status):
        raise NotImplementedError

    def _eval(self, x, inverse, status):
        """(z, logdet) with logdet written by the kernels (no autograd)."""
        logdet = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
        with torch.no_grad():
            z = self._run(x, inverse, logdet, K_.MODE_WRITE, status)
        return z, logdet

    def _call(self, x, inverse, status=None):
        """Run the layer; with ``status`` given the caller checks it later."""
        x = _check_input(x)
        st = status
        if st is None and self._n_status:
            st = torch.zeros(self._n_status, dtype=torch.int32, device=x.device)
        if _needs_grad(self, x):
            named = self._named_param_list()
            z, logdet = _LayerFn.apply(self, inverse, st, tuple(n for n, _ in named), x,
                                       *(t for _, t in named))
        else:
            z, logdet = self._eval(x, inverse, st)
        if status is None and st is not None:
            check_status(st)
        return z, logdet


class FCNN(nn.Module):
    """Linear -> Tanh -> Linear -> Tanh -> Linear conditioner (flows.py:20-35)."""

    def __init__(self, in_dim, out_dim, hidden_dim):
        super().__init__()
        self.network = nn.Sequential(
            nn.Linear(in_dim, hidden_dim), nn.Tanh(),
            nn.Linear(hidden_dim, hidden_dim), nn.Tanh(),
            nn.Linear(hidden_dim, out_dim))

    def forward(self, x):
        return self.network(x)


_HOST = []


_DERIVED_STATE = ("_pack_cache", "_winv_key", "_vjp_cache", "_ar_tree", "_named_cache", "_ar_names", "_wide_cache")


def _host_helper():
    """The host helper extension (csrc/nfk_host.cpp, built by build()), or None
    (then the caches are validated in Python: same keys, slower)."""
    if not _HOST:
        try:
            from . import _nfk_host as hs  # noqa: F401
        except ImportError:
            hs = None
        _HOST.append(hs)
    return _HOST[0]


def _is_stock_fcnn(net):
    if type(net) is not FCNN:
        return False
    n = net.network
    return (len(n) == 5 and all(isinstance(n[i], nn.Linear) for i in (0, 2, 4))
            and all(isinstance(n[i], nn.Tanh) for i in (1, 3)))


def _vjp_out(names, need, gx, grads):
    """_LayerFn.backward's result list: dL/dx (if wanted), then per parameter."""
    return [gx if need[0] else None] + [grads.get(n) if r else None for n, r in zip(names, need[1:])]


def _dense(g, like):
    return torch.zeros_like(like) if g is None else g.contiguous()


@functools.lru_cache(maxsize=None)
def _rnvp_fused_half(h, hidden):
    if K_.fused_realnvp_supported(h, hidden):
        return h
    hp = (h + 15) // 16 * 16
    return hp if K_.fused_realnvp_supported(hp, hidden) else None


def rnvp_pad(x, h, hp):
    """[B, 2h] -> [B, 2hp]: the halves at columns [0, h) and [hp, hp + h), zeros
    elsewhere (x itself when hp == h)."""
    if hp == h:
        return x
    xp = torch.zeros(x.shape[0], 2 * hp, dtype=x.dtype, device=x.device)
    xp[:, :h] = x[:, :h]
    xp[:, hp:hp + h] = x[:, h:]
    return xp


def rnvp_unpad(zp, h, hp):
    """Inverse of rnvp_pad."""
    if hp == h:
        return zp
    return torch.cat([zp[:, :h], zp[:, hp:hp + h]], 1)


class RealNVP(_HipFlow):
    """Affine coupling, two halves per layer (flows.py:38-76).

    forward:  up <- t1(lo) + up*exp(s1(lo));  lo <- t2(up) + lo*exp(s2(up))
    inverse:  lo <- (lo - t2(up))*exp(-s2(up));  up <- (up - t1(lo))*exp(-s1(lo))
    """

    def __init__(self, dim, hidden_dim=800, base_network=FCNN):
        super().__init__()
        self.dim = dim
        self.t1 = base_network(dim // 2, dim // 2, hidden_dim)
        self.s1 = base_network(dim // 2, dim // 2, hidden_dim)
        self.t2 = base_network(dim // 2, dim // 2, hidden_dim)
        self.s2 = base_network(dim // 2, dim // 2, hidden_dim)
        self._pack_cache = None

    def _fused_half(self, hidden):
        """Half-dimension the fused kernel runs this layer at: dim // 2 when the
        kernel takes it, else the next multiple of 16 it takes (the halves
        zero-padded: padded inputs meet zero weight columns and the padded s, t
        outputs are exactly 0, so z and log|det| are unchanged), else None."""
        return _rnvp_fused_half(self.dim // 2, hidden)

    def _fused_pack(self, device):
        """Weights of the four conditioners re-packed for nfk_fused_realnvp;
        rebuilt when any weight changes (None when the fused kernel does not apply)."""
        nets = (self.s1, self.t1, self.s2, self.t2)
        if not config.USE_FUSED or not all(_is_stock_fcnn(n) for n in nets):
            return None
        h = self.dim // 2
        hidden = self.s1.network[0].out_features
        if any(n.network[0].out_features != hidden for n in nets):
            return None
        hp = self._fused_half(hidden)
        if hp is None or torch.device(device).type != "cuda":
            return None
        params = [t for n in nets for i in (0, 2, 4) for t in (n.network[i].weight, n.network[i].bias)]
        if any(p.device != device or p.dtype != torch.float32 for p in params):
            return None
        key = tuple((p.data_ptr(), p._version) for p in params)
        if self._pack_cache is not None and self._pack_cache[0] == key:
            return self._pack_cache[1]
        if hp != h:
            # zero-padded first-layer input columns, last-layer output rows and biases
            padded = []
            for j, t in enumerate(params):
                t = t.detach()
                if j % 6 == 0:    # W0 [H, h]
                    t = torch.nn.functional.pad(t, (0, hp - h))
                elif j % 6 == 4:  # W4 [h, H]
                    t = torch.nn.functional.pad(t, (0, 0, 0, hp - h))
                elif j % 6 == 5:  # b4 [h]
                    t = torch.nn.functional.pad(t, (0, hp - h))
                padded.append(t)
            params = padded
        pack = K_.fused_realnvp_pack(params, hp, hidden)
        self._pack_cache = (key, pack, hidden, hp)
        return pack

    def _wide_pack(self, device, batch):
        """The K_.WideRnvpPack of nfk_wide_rnvp -- the layer as a weight stream
        (Polymer_rnvp.yaml's RealNVP(2048, hidden 4000) at its 40-row batches):
        every Linear of the four conditioners packed once (nfk_wlin_pack),
        rebuilt when any parameter changes; None when it does not apply (non-stock
        conditioners, unequal hidden widths, an unsupported shape, or a batch
        above config.WIDE_RNVP_MAX_ROWS, where library GEMMs are compute-bound
        and faster)."""
        if not config.USE_WIDE_RNVP or batch > config.WIDE_RNVP_MAX_ROWS or self.dim % 2:
            return None
        c = self.__dict__.get("_wide_cache")
        if c is not None and c[2] is not None and c[3] == device and c[2].valid():
            # the cached key's watch (csrc/nfk_host.cpp make_watch: the module
            # tree's dicts and the 24 tensors' storage and version, ~2 us) instead
            # of walking the modules (~60-150 us per call, the layer's launch time)
            return c[1]
        nets = (self.s1, self.t1, self.s2, self.t2)
        if torch.device(device).type != "cuda" or not all(_is_stock_fcnn(n) for n in nets):
            return None
        hidden = self.s1.network[0].out_features
        if any(n.network[0].out_features != hidden for n in nets) or not K_.wide_rnvp_supported(self.dim // 2,
                                                                                                 hidden):
            return None
        # pack index 6 c + 2 l + g: c = 0 (s1, t1) / 1 (s2, t2), l = Linear 0/2/4, g = s/t
        order = [(n, i) for c in ((self.s1, self.t1), (self.s2, self.t2)) for i in (0, 2, 4) for n in c]
        params = [t for n, i in order for t in (n.network[i].weight, n.network[i].bias)]
        if any(p.device != device or p.dtype != torch.float32 for p in params):
            return None
        key = tuple((p.data_ptr(), p._version) for p in params)
        if c is not None and c[0] == key:
            wp = c[1]
        else:
            packs = [K_.wlin_pack(n.network[i].weight) for n, i in order]
            biases = [n.network[i].bias.detach().contiguous() for n, i in order]
            wp = K_.WideRnvpPack(packs, biases, self.dim // 2, hidden)
        watch = None
        hs = _host_helper()
        if hs is not None:
            dicts = [self.__dict__["_modules"]]
            for n in nets:
                net = n.__dict__["_modules"]["network"]
                dicts += [n.__dict__["_modules"], net.__dict__["_modules"]]
                dicts += [net.__dict__["_modules"][str(i)].__dict__["_parameters"] for i in (0, 2, 4)]
            watch = hs.make_watch(dicts, params)
        self.__dict__["_wide_cache"] = (key, wp, watch, device)
        return wp

    def _chain_shape(self, device):
        """("rnvp", kernel half_dim, hidden, half_dim) when this layer runs as the
        fused kernel and the chain form applies (so it may join an
        nfk_fused_realnvp_chain launch with layers of the same shape), else None."""
        if self.dim % 2 or self._fused_pack(device) is None:
            return None
        hidden, hp = self._pack_cache[2], self._pack_cache[3]
        return ("rnvp", hp, hidden, self.dim // 2) if K_.fused_realnvp_chain_max(hp, hidden) > 0 else None

    def _run(self, x, inverse, logdet, mode, status):
        h = self.dim // 2
        if x.shape[1] != self.dim or self.dim - h != h:
            # the reference fails the same way (shape broadcast in flows.py:56)
            raise RuntimeError("RealNVP needs an even feature dimension equal to dim=%d (got %d)"
                               % (self.dim, x.shape[1]))
        pack = self._fused_pack(x.device)
        if pack is not None:
            hidden, hp = self._pack_cache[2], self._pack_cache[3]
            xk = rnvp_pad(x, h, hp)
            zk = torch.empty_like(xk, memory_format=torch.contiguous_format)
            K_.fused_realnvp(xk, pack, hp, hidden, zk, logdet=logdet, logdet_mode=mode, inverse=inverse)
            return rnvp_unpad(zk, h, hp)
        wide = self._wide_pack(x.device, x.shape[0])
        if wide is not None:
            z = torch.empty_like(x, memory_format=torch.contiguous_format)
            xc = x if x.stride(1) == 1 else x.contiguous()
            K_.wide_rnvp(xc, wide, z, logdet=logdet, logdet_mode=mode, inverse=inverse)
            return z
        z = torch.empty_like(x, memory_format=torch.contiguous_format)
        lo, up = x[:, :h], x[:, h:]
        zlo, zup = z[:, :h], z[:, h:]
        m2 = K_.MODE_ACC if mode != K_.MODE_NONE else K_.MODE_NONE
        if not inverse:
            s1, t1 = self.s1(lo), self.t1(lo)
            K_.affine_coupling(up, s1, t1, zup, logdet=logdet, logdet_mode=mode)
            s2, t2 = self.s2(zup), self.t2(zup)
            K_.affine_coupling(lo, s2, t2, zlo, logdet=logdet, logdet_mode=m2)
        else:
            s2, t2 = self.s2(up), self.t2(up)
            K_.affine_coupling(lo, s2, t2, zlo, logdet=logdet, logdet_mode=mode, inverse=True)
            s1, t1 = self.s1(zlo), self.t1(zlo)
            K_.affine_coupling(up, s1, t1, zup, logdet=logdet, logdet_mode=m2, inverse=True)
        return z

    _NETS = ("s1", "t1", "s2", "t2")

    def _vjp(self, x, names, params, gz, gld, inverse, need):
        """Backward by hand for four stock FCNN conditioners (else None: the
        generic autograd recompute): the conditioners recomputed and
        differentiated by fcnn_grad (GEMMs, split-K weight gradients), each
        affine half-coupling by nfk_affine_coupling_bwd (flows.py:52-76)."""
        want_names = {"%s.network.%d.%s" % (n, i, k) for n in self._NETS for i in (0, 2, 4)
                      for k in ("weight", "bias")}
        if not all(_is_stock_fcnn(getattr(self, n)) for n in self._NETS) or set(names) != want_names \
                or x.shape[1] != self.dim or self.dim % 2:
            return None
        h = self.dim // 2
        p = {n: t.detach() for n, t in zip(names, params)}
        want = {n for n, r in zip(names, need[1:]) if r}
        x = x.detach()
        B = x.shape[0]
        gz = torch.zeros_like(x) if gz is None else gz.contiguous()
        gldc = None if gld is None else gld.contiguous()
        grads = {}
        gx = torch.empty_like(x)

        # forward:  up' = t1(lo) + up e^{s1(lo)};  lo' = t2(up') + lo e^{s2(up')}
        # inverse:  lo' = (lo - t2(up)) e^{-s2(up)};  up' = (up - t1(lo')) e^{-s1(lo')}
        lo, up = x[:, :h], x[:, h:]
        order = (("s1", "t1", lo, up), ("s2", "t2", None, lo)) if not inverse else \
                (("s2", "t2", up, lo), ("s1", "t1", None, up))
        # recompute: the first half's conditioner input is an input half, the
        # second one's is the first half's output
        sn, tn, src, tgt = order[0]
        s_a, c_sa = fcnn_grad.forward_saved(p, sn + ".", src)
        t_a, c_ta = fcnn_grad.forward_saved(p, tn + ".", src)
        out_a = t_a + tgt * torch.exp(s_a) if not inverse else (tgt - t_a) * torch.exp(-s_a)
        sn2, tn2, _, tgt2 = order[1]
        s_b, c_sb = fcnn_grad.forward_saved(p, sn2 + ".", out_a)
        t_b, c_tb = fcnn_grad.forward_saved(p, tn2 + ".", out_a)
        # the second half-coupling's output half of z is its target (lo forward, up inverse)
        g_a_out = gz[:, h:] if not inverse else gz[:, :h]  # gradient reaching out_a from z
        g_b_out = gz[:, :h] if not inverse else gz[:, h:]
        gx_b = gx[:, :h] if not inverse else gx[:, h:]      # gradient slot of tgt2 (x half)
        gx_a = gx[:, h:] if not inverse else gx[:, :h]      # gradient slot of tgt (x half)
        g_s = torch.empty(B, h, dtype=x.dtype, device=x.device)
        g_t = torch.empty_like(g_s) if inverse else None
        K_.affine_coupling_bwd(tgt2, s_b, t_b, g_b_out, gldc, gx_b, g_s, g_t, inverse=inverse)
        g_tb = g_t if inverse else g_b_out
        g_in_b_s, gr = fcnn_grad.vjp(p, sn2 + ".", c_sb, g_s, True, want)
        grads.update(gr)
        g_in_b_t, gr = fcnn_grad.vjp(p, tn2 + ".", c_tb, g_tb, True, want)
        grads.update(gr)
        g_outa = g_a_out + g_in_b_s + g_in_b_t
        g_s2 = torch.empty_like(g_s)
        g_t2 = torch.empty_like(g_s) if inverse else None
        K_.affine_coupling_bwd(tgt, s_a, t_a, g_outa, gldc, gx_a, g_s2, g_t2, inverse=inverse)
        g_ta = g_t2 if inverse else g_outa
        g_src_s, gr = fcnn_grad.vjp(p, sn + ".", c_sa, g_s2, need[0], want)
        grads.update(gr)
        g_src_t, gr = fcnn_grad.vjp(p, tn + ".", c_ta, g_ta, need[0], want)
        grads.update(gr)
        if need[0]:
            g_src = gx[:, :h] if not inverse else gx[:, h:]  # src is lo forward, up inverse = gx_b's half
            g_src += g_src_s + g_src_t
        return [gx if need[0] else None] + [grads.get(n) for n in names]

    def forward(self, x):
        return self._call(x, False)

    def inverse(self, z):
        return self._call(z, True)


class _SplineMaps:
    """Device-resident int32 column maps of one coupling layer."""

    def __init__(self, lo_in, lo_out, up_in, up_out, device):
        mk = lambda v: torch.tensor(v, dtype=torch.int32, device=device)
        self.lo_in, self.lo_out = mk(lo_in), mk(lo_out)
        self.up_in, self.up_out = mk(up_in), mk(up_out)
        self.lo_in_long = self.lo_in.long()
        self.lists = (list(lo_in), list(lo_out), list(up_in), list(up_out))
        # (start, stride) when the lower input columns are an arithmetic
        # progression (every single-coordinate mask): x's lower columns are then
        # a strided view, read and written in place
        li = list(lo_in)
        st = li[1] - li[0] if len(li) > 1 else 1
        self.lo_prog = (li[0], st) if li and st > 0 and all(li[i] == li[0] + st * i for i in range(len(li))) \
            else None


class NSF_CL(_HipFlow):
    """Neural-spline coupling layer (flows.py:210-253).

    Per particle group of ``dim`` coordinates, ``mask`` selects the conditioning
    ("lower") coordinates; the others are transformed by a rational-quadratic
    spline whose (W, H, D) come from ``psi(lower)``.  The output places the
    masked coordinates first in every group (flows.py:239), exactly as the
    reference -- a non-prefix mask therefore permutes coordinates.
    """
    _n_status = 1

    def __init__(self, size, dim=3, K=32, B=3, hidden_dim=800, base_network=FCNN, device="cpu",
                 mask=[1]):
        super().__init__()
        self.size = size
        self.dim = dim
        self.K = K
        self.B = B
        self.device = device
        self.mask = torch.Tensor(mask).long()
        self.unmasked = torch.Tensor([x for x in range(self.dim) if x not in self.mask]).long()
        self.psi = base_network(len(mask) * self.size,
                                (3 * K - 1) * (self.dim - len(self.mask)) * self.size,
                                hidden_dim).to(self.device)
        self._maps_cache = {}
        self._pack_cache = None

    # column maps (x -> lower/upper, and where each lands in the output)
    def _maps(self, device):
        key = str(device)
        m = self._maps_cache.get(key)
        if m is None:
            mk, um = [int(v) for v in self.mask], [int(v) for v in self.unmasked]
            nm = len(mk)
            lo_in = [p * self.dim + c for p in range(self.size) for c in mk]
            up_in = [p * self.dim + c for p in range(self.size) for c in um]
            lo_out = [p * self.dim + i for p in range(self.size) for i in range(nm)]
            up_out = [p * self.dim + nm + i for p in range(self.size) for i in range(len(um))]
            m = self._maps_cache[key] = _SplineMaps(lo_in, lo_out, up_in, up_out, device)
        return m

    def _fused_pack(self, device):
        """Weights re-packed for the fused kernel; rebuilt when any weight changes."""
        if not config.USE_FUSED or not _is_stock_fcnn(self.psi):
            return None
        lins = [self.psi.network[i] for i in (0, 2, 4)]
        n_lo, n_up = len(self.mask) * self.size, len(self.unmasked) * self.size
        hidden = lins[0].out_features
        if not K_.fused_nsf_supported(n_lo, n_up, hidden, self.K):
            return None
        params = [t for l in lins for t in (l.weight, l.bias)]
        if any(p.device != device or p.dtype != torch.float32 for p in params):
            return None
        key = tuple((p.data_ptr(), p._version) for p in params)
        if self._pack_cache is not None and self._pack_cache[0] == key:
            return self._pack_cache[1]
        pack = K_.fused_nsf_pack(*params, n_lo, n_up, hidden, self.K)
        self._pack_cache = (key, pack, hidden)
        return pack

    def _vjp_pack(self, device):
        """The fused backward's pack (nfk_fused_nsf_vjp_pack), rebuilt when any
        weight changes; None when that kernel does not apply."""
        if not (config.USE_FUSED and config.USE_FUSED_VJP) or not _is_stock_fcnn(self.psi):
            return None
        lins = [self.psi.network[i] for i in (0, 2, 4)]
        n_lo, n_up = len(self.mask) * self.size, len(self.unmasked) * self.size
        hidden = lins[0].out_features
        if not K_.fused_nsf_vjp_supported(n_lo, n_up, hidden, self.K):
            return None
        params = [t for l in lins for t in (l.weight, l.bias)]
        if any(p.device != device or p.dtype != torch.float32 for p in params):
            return None
        key = tuple((p.data_ptr(), p._version) for p in params)
        cache = self.__dict__.get("_vjp_cache")
        if cache is not None and cache[0] == key:
            return cache[1]
        pack = K_.fused_nsf_vjp_pack(*params, n_lo, n_up, hidden, self.K)
        self.__dict__["_vjp_cache"] = (key, pack, hidden)
        return pack

    def _chain_shape(self, device):
        """(n_lo, n_up, hidden, K, B) when this layer runs as the fused kernel
        (so it may join an nfk_fused_nsf_chain launch with layers of the same
        shape), else None."""
        if self._fused_pack(device) is None:
            return None
        return (len(self.mask) * self.size, len(self.unmasked) * self.size, self._pack_cache[2], self.K,
                float(self.B))

    def _run(self, x, inverse, logdet, mode, status):
        if x.shape[1] != self.size * self.dim:
            raise RuntimeError("NSF_CL(size=%d, dim=%d) got %d features"
                               % (self.size, self.dim, x.shape[1]))
        maps = self._maps(x.device)
        z = torch.empty_like(x, memory_format=torch.contiguous_format)
        pack = self._fused_pack(x.device)
        if pack is not None:
            K_.fused_nsf(x, pack, maps.up_in, maps.up_out, maps.lo_in, maps.lo_out,
                         self._pack_cache[2], z, logdet=logdet, logdet_mode=mode, K=self.K,
                         tail_bound=self.B, inverse=inverse, status=status)
            return z
        lower = x.index_select(1, maps.lo_in_long)
        params = self.psi(lower).contiguous()
        b = float(self.B)
        K_.rqs_coupling(x, params, maps.up_in, maps.up_out, z, lo_in=maps.lo_in,
                        lo_out=maps.lo_out, logdet=logdet, logdet_mode=mode, K=self.K,
                        left=-b, right=b, bottom=-b, top=b, tails=True, param_mode=0,
                        inverse=inverse, status=status)
        return z

    def _vjp(self, x, names, params, gz, gld, inverse, need):
        """Backward: the conditioner is recomputed and, for the stock FCNN,
        differentiated by hand (fcnn_grad: hipBLASLt GEMMs, the weight
        gradients split over the batch), any other one by torch autograd; the
        spline by nfk_rqs_coupling_bwd."""
        maps = self._maps(x.device)
        # stock FCNN: recompute and differentiate by hand (fcnn_grad: split-K
        # weight gradients); any other conditioner through autograd
        manual = _is_stock_fcnn(self.psi) and set(names) == set(
            "psi.network.%d.%s" % (i, k) for i in (0, 2, 4) for k in ("weight", "bias"))
        rows_ok = config.FUSED_VJP_MAX_ROWS is None or x.shape[0] <= config.FUSED_VJP_MAX_ROWS
        vpack = self._vjp_pack(x.device) if manual and rows_ok else None
        if vpack is not None:
            # fused: the conditioner recomputed on the matrix cores and the
            # spline VJP in one kernel (nfk_fused_nsf_vjp); it hands over
            # dL/dparams and the activations [h | 1] for the GEMMs below
            x = x.detach().contiguous()
            B, H = x.shape[0], self.__dict__["_vjp_cache"][2]
            ldh = (H + 4) // 4 * 4
            hbuf = torch.empty(2, B, ldh, dtype=x.dtype, device=x.device)
            gp = torch.empty(B, len(maps.lists[2]) * (3 * self.K - 1), dtype=x.dtype, device=x.device)
            gx = torch.empty_like(x)
            K_.fused_nsf_vjp(x, vpack, maps.up_in, maps.up_out, maps.lo_in, maps.lo_out, H,
                             None if gz is None else gz.contiguous(), None if gld is None else gld.contiguous(),
                             gp, gx, hbuf[0], hbuf[1], K=self.K, tail_bound=float(self.B), inverse=inverse)
            pmap = {n: t.detach() for n, t in zip(names, params)}
            want = {n for n, r in zip(names, need[1:]) if r}
            n_lo = len(maps.lists[0])
            if maps.lo_prog is not None:
                # dL/dx of the lower columns added in place (a strided view) by
                # the last input-gradient GEMM
                a, st = maps.lo_prog
                into = gx[:, a::st][:, :n_lo] if need[0] else None
            else:
                into = None
            # the first Linear's weight and bias gradients in one GEMM against
            # [lower | 1], gathered by one kernel (a strided view of x made the
            # library GEMM copy it, and the bias gradient was a column sum)
            l0 = ("psi.network.0.weight", "psi.network.0.bias")
            if any(n in want for n in l0) or maps.lo_prog is None:
                lower = K_.gather_cols_ones(x, maps.lo_in)
            else:
                lower = x[:, :0]  # (unused: no first-Linear gradient wanted)
            g_lower, grads = fcnn_grad.vjp(pmap, "psi.", (lower, hbuf[0][:, :H + 1], hbuf[1][:, :H + 1]),
                                           gp, need[0], want, gx_into=into)
            if g_lower is not None:
                gx.index_add_(1, maps.lo_in_long, g_lower)
            return [gx if need[0] else None] + [grads.get(n) for n in names]
        if manual:
            lower = x.detach().index_select(1, maps.lo_in_long)
            pmap = {n: t.detach() for n, t in zip(names, params)}
            raw, cache = fcnn_grad.forward_saved(pmap, "psi.", lower)
        else:
            with torch.enable_grad():
                lower = x.detach().index_select(1, maps.lo_in_long).requires_grad_(need[0])
                pd = {n: t.detach().requires_grad_(r) for n, t, r in zip(names, params, need[1:])}
                raw = torch_math.conditioner(self, pd, "psi", lower)
        rawc = raw.detach().contiguous()
        gp = torch.empty_like(rawc)
        gx = torch.empty(x.shape, dtype=x.dtype, device=x.device)
        b = float(self.B)
        K_.rqs_coupling_bwd(x, rawc, maps.up_in, maps.up_out,
                            None if gz is None else gz.contiguous(),
                            None if gld is None else gld.contiguous(), gp, gx, lo_in=maps.lo_in,
                            lo_out=maps.lo_out, K=self.K, left=-b, right=b, bottom=-b, top=b,
                            tails=True, param_mode=0, inverse=inverse)
        if manual:
            want = {n for n, r in zip(names, need[1:]) if r}
            g_lower, grads = fcnn_grad.vjp(pmap, "psi.", cache, gp, need[0], want)
            if g_lower is not None:
                gx.index_add_(1, maps.lo_in_long, g_lower)
            return [gx if need[0] else None] + [grads.get(n) for n in names]
        inputs = [t for t in [lower] + list(pd.values()) if t.requires_grad]
        got = list(torch.autograd.grad(raw, inputs, gp, allow_unused=True)) if inputs else []
        g_lower = got.pop(0) if need[0] else None
        if g_lower is not None:
            gx.index_add_(1, maps.lo_in_long, g_lower)
        out = [gx if need[0] else None]
        for t in pd.values():
            out.append(got.pop(0) if t.requires_grad else None)
        return out

    def forward(self, x):
        return self._call(x, False)

    def inverse(self, z):
        return self._call(z, True)


class NSF_AR(_HipFlow):
    """Autoregressive neural-spline flow (flows.py:152-209).

    Coordinate i is splined with (W, H, D) = layers[i-1](cos/sin(pi*v[:, :i]/B))
    (``init_param`` for i = 0), where v is the input in ``forward`` and the
    already-inverted output in ``inverse`` (flows.py:201).
    """

    def __init__(self, dim, K=32, B=3, hidden_dim=800, base_network=FCNN, device="cpu"):
        super().__init__()
        self.dim = dim
        self.K = K
        self.B = B
        self.device = device
        self.layers = nn.ModuleList()
        # registered as a Parameter on every device (the reference's `.to(device)`
        # drops the registration for non-CPU devices, flows.py:164)
        self.init_param = nn.Parameter(torch.Tensor(3 * K - 1))
        for i in range(1, dim):
            self.layers += [base_network(2 * i, 3 * K - 1, hidden_dim).to(self.device)]
        self.reset_parameters()
        self._cols = {}
        self._pack_cache = None
        self._ar_tree = None  # (module-tree fingerprint, the conditioners' Linear modules)

    @property
    def _n_status(self):
        return self.dim

    def _fused_pack(self, device):
        """The fused layer kernel's pack (nfk_fused_ar: every conditioner and
        spline of the layer in one launch), rebuilt when any parameter
        changes; None when it does not apply (non-stock conditioners, unequal
        hidden widths, an unsupported shape).

        Per call this only fingerprints the module tree (object ids, read from
        the modules' own dicts) and the parameters (storage, version): at the
        applications' dim 96 a layer has 95 conditioners and 571 tensors, and
        walking them through nn.Module attribute access cost more host time
        than the whole launch at their 40-row batches."""
        if not config.USE_FUSED or self.dim < 2:
            return None
        hs = _host_helper()
        if hs is not None and self._pack_cache is not None and self._pack_cache[4] is not None:
            # the same key kept in C++ (csrc/nfk_host.cpp): a watch over every
            # dict of the module tree (CPython's dict version tags) and every
            # parameter (storage, version) -- ~20 us at Polymer's 2,047
            # conditioners, where recomputing the key in Python took ~23 ms --
            # else the key's hash recomputed in C++ (~1 ms)
            hdev, hw = self._pack_cache[4]
            if hdev == device:
                if isinstance(hw, int):
                    if hw == hs.ar_state(self.layers._modules, self.init_param, FCNN, nn.Linear, nn.Tanh):
                        return self._pack_cache[1]
                elif hw.valid():
                    return self._pack_cache[1]
        lin = self._stock_linears()
        if not lin:
            return None
        params = [self.init_param]
        for m in lin:
            pp = m.__dict__["_parameters"]
            params.append(pp.get("weight"))
            params.append(pp.get("bias"))
        if any(p is None for p in params):
            return None
        key = (device, tuple((p.data_ptr(), p._version) for p in params))
        if self._pack_cache is not None and self._pack_cache[0] == key:
            return self._pack_cache[1]
        hidden = lin[0].out_features
        if any(m.out_features != hidden for m in lin[0::3]) or not K_.fused_ar_supported(self.dim, hidden, self.K):
            return None
        if any(p.device != device or p.dtype != torch.float32 for p in params):
            return None
        ws = [tuple(params[1 + 6 * i:7 + 6 * i]) for i in range(self.dim - 1)]
        pack, keep = K_.fused_ar_pack(ws, self.init_param, self.dim, hidden, self.K)
        hkey = None
        if hs is not None:
            hw = hs.ar_watch(self.__dict__["_parameters"], self.__dict__["_modules"], self.layers._modules,
                             self.init_param, FCNN, nn.Linear, nn.Tanh)
            if hw is None:
                hw = hs.ar_state(self.layers._modules, self.init_param, FCNN, nn.Linear, nn.Tanh)
                hw = hw if hw >= 0 else None
            hkey = (device, hw) if hw is not None else None
        self._pack_cache = (key, pack, hidden, keep, hkey)
        return pack

    def reset_parameters(self):
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
        pack = self._fused_pack(x.device)
        if pack is not None and inverse and not K_.fused_ar_inverse_supported(self.dim, self._pack_cache[2], self.K):
            # a streamed-forward shape (Polymer's 2,048 coordinates): the inverse
            # column by column, one launch per column issued by the library
            hidden, keep = self._pack_cache[2], self._pack_cache[3]
            if config.USE_AR_SEQINV and K_.ar_seqinv_supported(self.dim, hidden, self.K):
                z = torch.empty_like(x, memory_format=torch.contiguous_format)
                K_.ar_seqinv(x, keep[3], keep[1], self.dim, hidden, self.K, float(self.B), z, logdet=logdet,
                             logdet_mode=mode, status=status)
                return z
            pack = None  # (the per-column path below)
        if pack is not None:
            z = torch.empty_like(x, memory_format=torch.contiguous_format)
            K_.fused_ar(x, pack, self.dim, self._pack_cache[2], self.K, float(self.B), z, logdet=logdet,
                        logdet_mode=mode, inverse=inverse, status=status)
            return z
        z = torch.zeros_like(x, memory_format=torch.contiguous_format)
        cond = z if inverse else x
        b = float(self.B)
        for i in range(self.dim):
            if i == 0:
                params = self.init_param.detach().to(torch.float32).expand(n, -1).contiguous()
            else:
                params = self.layers[i - 1](self.trig_transform(cond[:, :i])).contiguous()
            m = mode if (i == 0 or mode == K_.MODE_NONE) else K_.MODE_ACC
            col = self._col(i, x.device)
            K_.rqs_coupling(x, params, col, col, z, logdet=logdet, logdet_mode=m, K=self.K,
                            left=-b, right=b, bottom=-b, top=b, tails=True, param_mode=0,
                            inverse=inverse,
                            status=None if status is None else status[i:i + 1])
        return z

    def _vjp(self, x, names, params, gz, gld, inverse, need):
        """Backward by hand for stock FCNN conditioners (else None: autograd
        recompute).  Column i: the spline VJP (nfk_rqs_coupling_bwd), then the
        conditioner's (fcnn_grad) and the trig features' (nfk_trig_features_bwd)
        into the gradient of the coordinates it read -- x[:, :i] forward, the
        output z[:, :i] inverse (flows.py:174-209), so the inverse runs the
        columns last to first, each one's output gradient complete."""
        lin = self._stock_linears() if self.dim >= 2 else []
        if (self.dim >= 2 and not lin) or x.shape[1] != self.dim:
            return None
        if not inverse and self.dim >= 2 and len(names) == 1 + 6 * (self.dim - 1) \
                and set(names) == self._ar_name_set():
            H = lin[0].out_features
            n, P = self.dim - 1, 3 * self.K - 1
            # peak bytes of the batched backward per (conditioner, row): h1, h2,
            # the tanh-derivative temporaries and ga1/ga2 with theirs (8 H), the
            # logits, their gradient and its transposed copy (3 P), the expanded
            # trig features bmm materialises and the feature-gradient product (4 n)
            per = 4 * n * x.shape[0] * (8 * H + 3 * P + 4 * n)
            per += 2 * 4 * n * H * 2 * n  # the zero-padded first-Linear stack and its gradient
            if all(m.out_features == H for m in lin[0::3]) and per <= config.AR_BATCHED_VJP_BYTES:
                return self._vjp_batched(x, names, params, gz, gld, need, H)
        p = {n: t.detach() for n, t in zip(names, params)}
        want = {n for n, r in zip(names, need[1:]) if r}
        x = x.detach()
        B, b = x.shape[0], float(self.B)
        cond = self._eval(x, True, None)[0] if inverse else x
        gout = _dense(gz, x).clone() if inverse else _dense(gz, x)
        gldc = None if gld is None else gld.contiguous()
        gx = torch.empty_like(x)
        grads = {}
        order = range(self.dim - 1, -1, -1) if inverse else range(self.dim)
        for i in order:
            if i == 0:
                prm = p["init_param"].to(torch.float32).expand(B, -1).contiguous()
            else:
                prm, cache = fcnn_grad.forward_saved(p, "layers.%d." % (i - 1), self.trig_transform(cond[:, :i]))
            gprm = torch.empty_like(prm)
            col = self._col(i, x.device)
            K_.rqs_coupling_bwd(x, prm, col, col, gout, gldc, gprm, gx, K=self.K, left=-b, right=b,
                                bottom=-b, top=b, tails=True, param_mode=0, inverse=inverse)
            if i == 0:
                if "init_param" in want:
                    grads["init_param"] = gprm.sum(0)
                continue
            gfeat, gr = fcnn_grad.vjp(p, "layers.%d." % (i - 1), cache, gprm, True, want)
            grads.update(gr)
            K_.trig_features_bwd(cond[:, :i], gfeat, gout if inverse else gx, b)
        return _vjp_out(names, need, gx, grads)

    def _stock_linears(self):
        """The conditioners' Linear modules in order (3 per conditioner) when
        every conditioner is the stock FCNN, else []; cached on a fingerprint of
        the module tree (object ids read from the modules' own dicts)."""
        mods = []
        for n in self.layers._modules.values():
            net = n.__dict__["_modules"].get("network")
            mods.append(n)
            mods.append(net)
            if net is not None:
                mods.extend(net.__dict__["_modules"].values())
        tree = tuple(map(id, mods))
        if self._ar_tree is not None and self._ar_tree[0] == tree:
            return self._ar_tree[1]
        lin = [n.network[j] for n in self.layers for j in (0, 2, 4)] \
            if all(_is_stock_fcnn(n) for n in self.layers) else []
        # the fingerprinted modules are kept alive with it, so none of their ids
        # can be reused by a replacement module while the entry stands
        self._ar_tree = (tree, lin, mods)
        return lin

    def _named_param_list(self):
        """named_parameters() of the layer, cached on the module tree and the
        parameter objects (ids read from the modules' own dicts): at dim 96 a
        walk through nn.Module's generators cost ~1.5 ms of host time per call."""
        if self.__dict__["_parameters"].keys() != {"init_param"}:
            return list(self.named_parameters())
        fp = [id(self.__dict__["_parameters"]["init_param"])]
        for n in self.layers._modules.values():
            fp.append(id(n))
            for m in n.__dict__["_modules"].values():
                fp.append(id(m))
                for sub in m.__dict__["_modules"].values():
                    fp.append(id(sub))
                    fp.extend(map(id, sub.__dict__["_parameters"].values()))
                fp.extend(map(id, m.__dict__["_parameters"].values()))
            fp.extend(map(id, n.__dict__["_parameters"].values()))
        fp = tuple(fp)
        c = self.__dict__.get("_named_cache")
        if c is None or c[0] != fp:
            c = self.__dict__["_named_cache"] = (fp, list(self.named_parameters()))
        return c[1]

    def _ar_name_set(self):
        c = self.__dict__.get("_ar_names")
        if c is None:
            c = self.__dict__["_ar_names"] = frozenset(
                ["init_param"] + ["layers.%d.network.%d.%s" % (i, j, k) for i in range(self.dim - 1)
                                  for j in (0, 2, 4) for k in ("weight", "bias")])
        return c

    def _w1_index(self, H, device):
        """Flat positions, in the zero-padded [dim-1, H, 2 (dim-1)] stack of the
        conditioners' first-Linear weights, of each conditioner's W1 [H, 2i]
        elements in order: its cos column c -> padded column c, its sin column
        i + c -> padded column (dim - 1) + c (trig_transform's cat(cos, sin),
        flows.py:172-173, over all dim - 1 leading coordinates)."""
        key = ("w1idx", H, str(device))
        idx = self._cols.get(key)
        if idx is None:
            n = self.dim - 1
            parts = []
            for i in range(1, self.dim):
                c = torch.arange(2 * i)
                col = torch.where(c < i, c, (n - i) + c)  # sin column i + c' -> n + c'
                rows = torch.arange(H)[:, None] * (2 * n) + col[None, :]
                parts.append(((i - 1) * H * 2 * n + rows).reshape(-1))
            idx = self._cols[key] = torch.cat(parts).to(device)
        return idx

    def _vjp_batched(self, x, names, params, gz, gld, need, H):
        """Forward-direction backward of the whole layer at once.  The dim - 1
        conditioners are independent given x (flows.py:182-189), so their
        recompute and backward are batched GEMMs over a stack of the
        conditioners' weights (the first Linear zero-padded to all 2 (dim - 1)
        trig features, so conditioner i still sees only x[:, :i]); the spline
        VJP of every column is one nfk_rqs_coupling_bwd launch; the trig
        features' backward one nfk_trig_features_bwd over the summed feature
        gradients.  A few dozen launches instead of ~20 per column: the
        applications train this layer on 40-50 rows, where launches are the
        cost.  Same values as the per-column path up to fp32 summation order."""
        p = {nm: t.detach() for nm, t in zip(names, params)}
        want = {nm for nm, r in zip(names, need[1:]) if r}
        x = x.detach().contiguous()
        B, D, n, P, b = x.shape[0], self.dim, self.dim - 1, 3 * self.K - 1, float(self.B)
        pre = ["layers.%d.network." % i for i in range(n)]
        W1 = torch.cat([p[q + "0.weight"].reshape(-1) for q in pre])
        idx = self._w1_index(H, x.device)
        W1p = torch.zeros(n * H * 2 * n, dtype=x.dtype, device=x.device)
        W1p[idx] = W1
        W1p = W1p.view(n, H, 2 * n)
        b1 = torch.stack([p[q + "0.bias"] for q in pre])
        W2 = torch.stack([p[q + "2.weight"] for q in pre])
        b2 = torch.stack([p[q + "2.bias"] for q in pre])
        W3 = torch.stack([p[q + "4.weight"] for q in pre])
        b3 = torch.stack([p[q + "4.bias"] for q in pre])
        feat = self.trig_transform(x[:, :n])                               # [B, 2n]
        fb = feat.unsqueeze(0).expand(n, B, 2 * n)
        h1 = torch.tanh(torch.baddbmm(b1.unsqueeze(1), fb, W1p.transpose(1, 2)))   # [n, B, H]
        h2 = torch.tanh(torch.baddbmm(b2.unsqueeze(1), h1, W2.transpose(1, 2)))
        out = torch.baddbmm(b3.unsqueeze(1), h2, W3.transpose(1, 2))              # [n, B, P]
        prm = torch.cat([p["init_param"].to(x.dtype).expand(B, 1, P), out.transpose(0, 1)], dim=1).contiguous()
        gprm = torch.empty_like(prm)
        gx = torch.empty_like(x)
        cols = self._col_range(x.device)
        K_.rqs_coupling_bwd(x, prm, cols, cols, _dense(gz, x), None if gld is None else gld.contiguous(), gprm,
                            gx, K=self.K, left=-b, right=b, bottom=-b, top=b, tails=True, param_mode=0,
                            inverse=False)
        grads = {}
        if "init_param" in want:
            grads["init_param"] = gprm[:, 0, :].sum(0)
        g3 = gprm[:, 1:, :].transpose(0, 1).contiguous()                   # [n, B, P]
        gW3, gb3 = torch.bmm(g3.transpose(1, 2), h2), g3.sum(1)
        ga2 = torch.bmm(g3, W3) * (1 - h2 * h2)
        gW2, gb2 = torch.bmm(ga2.transpose(1, 2), h1), ga2.sum(1)
        ga1 = torch.bmm(ga2, W2) * (1 - h1 * h1)
        gb1 = ga1.sum(1)
        gW1 = torch.bmm(ga1.transpose(1, 2), fb).reshape(-1)[idx] if any(q + "0.weight" in want for q in pre) \
            else None
        off = 0
        for i, q in enumerate(pre):
            if q + "0.weight" in want:
                sz = H * 2 * (i + 1)
                grads[q + "0.weight"] = gW1[off:off + sz].view(H, 2 * (i + 1))
            off += H * 2 * (i + 1)
            for nm, g in ((q + "0.bias", gb1[i]), (q + "2.weight", gW2[i]), (q + "2.bias", gb2[i]),
                          (q + "4.weight", gW3[i]), (q + "4.bias", gb3[i])):
                if nm in want:
                    grads[nm] = g
        if need[0]:
            gfeat = torch.bmm(ga1, W1p).sum(0)                             # [B, 2n]
            K_.trig_features_bwd(x[:, :n], gfeat, gx, b)
        return _vjp_out(names, need, gx, grads)

    def _col_range(self, device):
        key = ("all", str(device))
        c = self._cols.get(key)
        if c is None:
            c = self._cols[key] = torch.arange(self.dim, dtype=torch.int32, device=device)
        return c

    def forward(self, x):
        return self._call(x, False)

    def inverse(self, z):
        return self._call(z, True)


_NL_CODE = {torch.tanh: 0, F.leaky_relu: 1, F.elu: 2}


class Planar(_HipFlow):
    """Planar flow z = x + u_hat h(w.x + b) (flows_1.py:21-63)."""

    def __init__(self, dim, nonlinearity=torch.tanh):
        super().__init__()
        self.h = nonlinearity
        self.w = nn.Parameter(torch.Tensor(dim))
        self.u = nn.Parameter(torch.Tensor(dim))
        self.b = nn.Parameter(torch.Tensor(1))
        self.reset_parameters(dim)

    def reset_parameters(self, dim):
        init.uniform_(self.w, -math.sqrt(1 / dim), math.sqrt(1 / dim))
        init.uniform_(self.u, -math.sqrt(1 / dim), math.sqrt(1 / dim))
        init.uniform_(self.b, -math.sqrt(1 / dim), math.sqrt(1 / dim))

    def _run(self, x, inverse, logdet, mode, status):
        if inverse:
            raise NotImplementedError("Planar flow has no algebraic inverse.")
        if self.h not in _NL_CODE:
            raise NotImplementedError("Non-linearity is not supported.")
        z = torch.empty_like(x, memory_format=torch.contiguous_format)
        K_.planar(x, self.w.detach(), self.u.detach(), self.b.detach(), z, logdet=logdet,
                  logdet_mode=mode, nonlinearity=_NL_CODE[self.h])
        return z

    def _vjp(self, x, names, params, gz, gld, inverse, need):
        """Backward (nfk_planar_bwd): gx and the w, u, b gradients in one call."""
        if inverse or self.h not in _NL_CODE:
            return None
        p = {n: t.detach().contiguous() for n, t in zip(names, params)}
        x = x.detach()
        gx = torch.empty_like(x)
        grads = {"w": torch.empty_like(p["w"]), "u": torch.empty_like(p["u"]), "b": torch.empty_like(p["b"])}
        K_.planar_bwd(x, p["w"], p["u"], p["b"], None if gz is None else gz.contiguous(),
                      None if gld is None else gld.contiguous(), gx, grads["w"], grads["u"], grads["b"],
                      nonlinearity=_NL_CODE[self.h])
        return _vjp_out(names, need, gx, grads)

    def forward(self, x):
        return self._call(x, False)

    def inverse(self, z):
        raise NotImplementedError("Planar flow has no algebraic inverse.")


class Radial(_HipFlow):
    """Radial flow (flows_1.py:66-97).

    r = ||x - x0|| is the Frobenius norm over the WHOLE batch (flows_1.py:90),
    so outputs depend on the batch, and log_det has shape [1].  When the batch
    is sharded over ranks, set ``process_group`` (normalizingflow_amd.dist)
    and the squared norm is all-reduced so every shard sees the global r.
    The reference never initialises the parameters (its reset_parameters is
    broken); here they start at zero and ``reset_parameters(dim)`` works.
    """

    def __init__(self, dim):
        super().__init__()
        self.x0 = nn.Parameter(torch.zeros(dim))
        self.log_alpha = nn.Parameter(torch.zeros(1))
        self.beta = nn.Parameter(torch.zeros(1))
        self.process_group = None
        self._ws = {}

    def reset_parameters(self, dim):
        init.uniform_(self.x0, -math.sqrt(1 / dim), math.sqrt(1 / dim))
        init.uniform_(self.log_alpha, -math.sqrt(1 / dim), math.sqrt(1 / dim))
        init.uniform_(self.beta, -math.sqrt(1 / dim), math.sqrt(1 / dim))

    def _buffers_for(self, device):
        key = str(device)
        if key not in self._ws:
            self._ws[key] = (torch.empty(K_.radial_workspace_elems(), dtype=torch.float64,
                                         device=device),
                             torch.empty(1, dtype=torch.float64, device=device))
        return self._ws[key]

    def _run(self, x, inverse, logdet, mode, status, ld_scalar=None):
        if inverse:
            raise AttributeError("'Radial' object has no attribute 'inverse'")
        ws, sumsq = self._buffers_for(x.device)
        K_.radial_sumsq(x, self.x0.detach(), ws, sumsq)
        if self.process_group is not None:
            torch.distributed.all_reduce(sumsq, group=self.process_group)
        z = torch.empty_like(x, memory_format=torch.contiguous_format)
        if ld_scalar is None:
            ld_scalar = torch.empty(1, dtype=torch.float32, device=x.device)
        K_.radial_apply(x, self.x0.detach(), self.log_alpha.detach(), self.beta.detach(), sumsq,
                        z, ld_scalar, logdet=logdet, logdet_mode=mode)
        return z

    def _eval(self, x, inverse, status):
        ld = torch.empty(1, dtype=torch.float32, device=x.device)
        with torch.no_grad():
            z = self._run(x, inverse, None, K_.MODE_NONE, None, ld_scalar=ld)
        return z, ld

    def _vjp(self, x, names, params, gz, gld, inverse, need):
        """Backward (nfk_radial_bwd_scalars / _apply).  r is batch-global, so
        with a process group the recomputed sumsq is all-reduced as in the
        forward, and so is dL/dsumsq between the two calls (the backward of
        that all-reduce): every shard then sees the gradient of the global r."""
        if inverse:
            return None
        p = {n: t.detach().contiguous() for n, t in zip(names, params)}
        x = x.detach()
        B, D = x.shape
        ws, sumsq = self._buffers_for(x.device)
        K_.radial_sumsq(x, p["x0"], ws, sumsq)
        if self.process_group is not None:
            torch.distributed.all_reduce(sumsq, group=self.process_group)
        wsb = K_.flows_bwd_workspace(B, D, x.device)
        scal = torch.empty(4, dtype=torch.float32, device=x.device)
        gzc = None if gz is None else gz.contiguous()
        K_.radial_bwd_scalars(x, p["x0"], p["log_alpha"], p["beta"], sumsq, gzc,
                              None if gld is None else gld.reshape(1).contiguous(), scal, wsb)
        if self.process_group is not None:
            torch.distributed.all_reduce(scal[0:1], group=self.process_group)
        gx = torch.empty_like(x)
        gx0 = torch.empty_like(p["x0"])
        K_.radial_bwd_apply(x, p["x0"], gzc, scal, gx, gx0, wsb)
        grads = {"x0": gx0, "log_alpha": scal[1:2].clone(), "beta": scal[2:3].clone()}
        return _vjp_out(names, need, gx, grads)

    def forward(self, x):
        return self._call(x, False)


class MAF(_HipFlow):
    """Masked autoregressive flow (flows_1.py:159-195).

    Coordinate i is mapped by z_i = (x_i - mu_i) / exp(alpha_i) with
    (mu_i, alpha_i) = layers[i-1](x[:, :i]) (``initial_param`` for i = 0); the
    output is flipped along the features.  The forward conditioners all read
    x, so they run first and one nfk_maf launch maps every column; the inverse
    is sequential (column i conditions on the already-inverted columns).
    The reference allocates its log|det| on the CPU (flows_1.py:176), so it only
    runs on CPU tensors; here it runs on the device.
    """

    def __init__(self, dim, hidden_dim=8, base_network=FCNN):
        super().__init__()
        self.dim = dim
        self.layers = nn.ModuleList()
        self.initial_param = nn.Parameter(torch.Tensor(2))
        for i in range(1, dim):
            self.layers += [base_network(i, 2, hidden_dim)]
        self.reset_parameters()

    def reset_parameters(self):
        init.uniform_(self.initial_param, -math.sqrt(0.5), math.sqrt(0.5))

    def _run(self, x, inverse, logdet, mode, status):
        if x.shape[1] != self.dim:
            raise RuntimeError("MAF(dim=%d) got %d features" % (self.dim, x.shape[1]))
        out = torch.empty_like(x, memory_format=torch.contiguous_format)
        ip = self.initial_param.detach().to(torch.float32).contiguous()
        if not inverse:
            prm = (torch.cat([self.layers[i - 1](x[:, :i]) for i in range(1, self.dim)], dim=1)
                   if self.dim > 1 else None)
            K_.maf(x, ip, prm, out, 0, self.dim, logdet=logdet, logdet_mode=mode)
            return out
        K_.maf(x, ip, None, out, 0, 1, logdet=logdet, logdet_mode=mode, inverse=True)
        m2 = K_.MODE_ACC if mode != K_.MODE_NONE else K_.MODE_NONE
        for i in range(1, self.dim):
            prm = self.layers[i - 1](out[:, :i])
            K_.maf(x, ip, prm, out, i, i + 1, logdet=logdet, logdet_mode=m2, inverse=True)
        return out

    def _vjp(self, x, names, params, gz, gld, inverse, need):
        """Backward by hand for stock FCNN conditioners (else None: autograd
        recompute): nfk_maf_bwd for the affine steps, fcnn_grad for the
        conditioners, whose input gradient goes to x[:, :i] (forward) or to
        the output columns they read (inverse, run last column first)."""
        if not all(_is_stock_fcnn(n) for n in self.layers) or x.shape[1] != self.dim:
            return None
        p = {n: t.detach() for n, t in zip(names, params)}
        want = {n for n, r in zip(names, need[1:]) if r}
        x = x.detach()
        ip = p["initial_param"].to(torch.float32).contiguous()
        gldc = None if gld is None else gld.contiguous()
        gx = torch.empty_like(x)
        ginit = torch.empty(2, dtype=torch.float32, device=x.device)
        grads = {}
        cond = self._eval(x, True, None)[0] if inverse else x
        saved = [fcnn_grad.forward_saved(p, "layers.%d." % (i - 1), cond[:, :i].contiguous())
                 for i in range(1, self.dim)]
        if not inverse:
            prm = torch.cat([o for o, _ in saved], dim=1) if saved else None
            gprm = None if prm is None else torch.empty_like(prm)
            K_.maf_bwd(x, ip, prm, _dense(gz, x), gldc, 0, self.dim, gx, gprm, ginit)
            for i in range(1, self.dim):
                g_in, gr = fcnn_grad.vjp(p, "layers.%d." % (i - 1), saved[i - 1][1],
                                         gprm[:, 2 * (i - 1):2 * i].contiguous(), True, want)
                grads.update(gr)
                gx[:, :i] += g_in
        else:
            gout = _dense(gz, x).clone()
            for i in range(self.dim - 1, -1, -1):
                prm = saved[i - 1][0].contiguous() if i > 0 else None
                gprm = None if prm is None else torch.empty_like(prm)
                K_.maf_bwd(x, ip, prm, gout, gldc, i, i + 1, gx, gprm, ginit if i == 0 else None,
                           inverse=True)
                if i > 0:
                    g_in, gr = fcnn_grad.vjp(p, "layers.%d." % (i - 1), saved[i - 1][1], gprm, True, want)
                    grads.update(gr)
                    gout[:, :i] += g_in
        grads["initial_param"] = ginit
        return _vjp_out(names, need, gx, grads)

    def forward(self, x):
        return self._call(x, False)

    def inverse(self, z):
        return self._call(z, True)


class ActNorm(_HipFlow):
    """ActNorm (flows_1.py:198-215): z = x * exp(log_sigma) + mu; log|det| is
    the scalar sum(log_sigma) (shape [], broadcast by the model)."""

    def __init__(self, dim):
        super().__init__()
        self.dim = dim
        self.mu = nn.Parameter(torch.zeros(dim, dtype=torch.float))
        self.log_sigma = nn.Parameter(torch.zeros(dim, dtype=torch.float))

    def _launch(self, x, inverse, logdet, mode, ld_scalar):
        if x.shape[1] != self.dim:
            raise RuntimeError("ActNorm(dim=%d) got %d features" % (self.dim, x.shape[1]))
        z = torch.empty_like(x, memory_format=torch.contiguous_format)
        K_.actnorm(x, self.mu.detach(), self.log_sigma.detach(), z, logdet=logdet,
                   logdet_mode=mode, ld_scalar=ld_scalar, inverse=inverse)
        return z

    def _run(self, x, inverse, logdet, mode, status):
        return self._launch(x, inverse, logdet, mode, None)

    def _eval(self, x, inverse, status):
        ld = torch.empty((), dtype=torch.float32, device=x.device)
        with torch.no_grad():
            z = self._launch(x, inverse, None, K_.MODE_NONE, ld)
        return z, ld

    def _vjp(self, x, names, params, gz, gld, inverse, need):
        """Backward (nfk_actnorm_bwd); log|det| is the scalar +-sum(log_sigma)."""
        p = {n: t.detach().contiguous() for n, t in zip(names, params)}
        x = x.detach()
        gx = torch.empty_like(x)
        grads = {"mu": torch.empty_like(p["mu"]), "log_sigma": torch.empty_like(p["log_sigma"])}
        K_.actnorm_bwd(x, p["mu"], p["log_sigma"], _dense(gz, x), None if gld is None else gld.reshape(1).contiguous(),
                       gx, grads["mu"], grads["log_sigma"], inverse=inverse)
        return _vjp_out(names, need, gx, grads)

    def forward(self, x):
        return self._call(x, False)

    def inverse(self, z):
        return self._call(z, True)


class OneByOneConv(_HipFlow):
    """Invertible 1x1 convolution (flows_1.py:218-252): z = x @ P @ L @ (U + diag S).

    Same construction as the reference (QR of a numpy normal matrix, scipy LU),
    so a given ``np.random`` state yields the same P, L, S, U.  P is a
    non-persistent buffer (the reference keeps it as a plain attribute, so it
    is not in the state_dict either, but here it follows ``.to(device)``).  The
    products are plain GEMMs (hipBLASLt through torch.matmul) in the
    reference's association.  The inverse matrix is cached per weight version;
    the reference caches it once (``if not self.W_inv``, flows_1.py:244), which
    raises on its second call for dim > 1.
    """

    def __init__(self, dim):
        super().__init__()
        import scipy.linalg as sla
        self.dim = dim
        W, _ = sla.qr(np.random.randn(dim, dim))
        P, L, U = sla.lu(W)
        self.register_buffer("P", torch.tensor(P, dtype=torch.float), persistent=False)
        self.L = nn.Parameter(torch.tensor(L, dtype=torch.float))
        self.S = nn.Parameter(torch.tensor(np.diag(U), dtype=torch.float))
        self.U = nn.Parameter(torch.triu(torch.tensor(U, dtype=torch.float), diagonal=1))
        self.W_inv = None
        self._winv_key = None

    def _factors(self):
        eye = torch.diag(torch.ones(self.dim, device=self.L.device))
        L = torch.tril(self.L, diagonal=-1) + eye
        U = torch.triu(self.U, diagonal=1)
        return L, U + torch.diag(self.S)

    def _logdet_scalar(self, inverse):
        v = torch.sum(torch.log(torch.abs(self.S)))
        return -v if inverse else v

    def _z(self, x, inverse):
        if x.shape[1] != self.dim:
            raise RuntimeError("OneByOneConv(dim=%d) got %d features" % (self.dim, x.shape[1]))
        L, US = self._factors()
        if not inverse:
            return x @ self.P @ L @ US
        key = tuple((p.data_ptr(), p._version) for p in (self.P, self.L, self.S, self.U))
        if self.W_inv is None or self._winv_key != key:
            self.W_inv = torch.inverse(self.P @ L @ US)
            self._winv_key = key
        return x @ self.W_inv

    def _run(self, x, inverse, logdet, mode, status):
        z = self._z(x, inverse).contiguous()
        if mode != K_.MODE_NONE:
            ld = self._logdet_scalar(inverse)
            if mode == K_.MODE_ACC:
                logdet.add_(ld)
            else:
                logdet.copy_(ld.expand_as(logdet))
        return z

    def _eval(self, x, inverse, status):
        with torch.no_grad():
            return self._z(x, inverse).contiguous(), self._logdet_scalar(inverse)

    def _vjp(self, x, names, params, gz, gld, inverse, need):
        """Backward: the batch products are library GEMMs like the forward
        (dL/dx = gz W^T, dL/dW = x^T gz; W^-1 in the inverse), and only the
        [dim, dim] factorisation W = P L (U + diag S) is differentiated by
        autograd (parameter-sized, no batch dimension)."""
        p = {n: t.detach().requires_grad_(r) for n, t, r in zip(names, params, need[1:])}
        x = x.detach()
        gzc = _dense(gz, x)
        with torch.enable_grad():
            eye = torch.diag(torch.ones(self.dim, dtype=x.dtype, device=x.device))
            L = torch.tril(p["L"], diagonal=-1) + eye
            US = torch.triu(p["U"], diagonal=1) + torch.diag(p["S"])
            W = self.P.to(x.dtype) @ L @ US
            M = torch.inverse(W) if inverse else W
            gx = gzc @ M.t() if need[0] else None
            outs, gouts = [M], [x.t() @ gzc]
            if gld is not None:
                ld = torch.sum(torch.log(torch.abs(p["S"])))
                outs.append(-ld if inverse else ld)
                gouts.append(gld.reshape(()))
            wanted = [n for n in names if p[n].requires_grad]
            got = torch.autograd.grad(outs, [p[n] for n in wanted], gouts, allow_unused=True) if wanted else []
        return _vjp_out(names, need, gx, dict(zip(wanted, got)))

    def forward(self, x):
        return self._call(x, False)

    def inverse(self, z):
        return self._call(z, True)
