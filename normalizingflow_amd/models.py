"""NormalizingFlowModel with the reference's API (nf/models.py:5-40).

forward(x)  -> (z, prior_logprob, log_det)      models.py:13-20
inverse(z)  -> (x, log_det)                     models.py:22-29
sample(n)   -> (x.data, log_px.data, z.data)    models.py:31-35
evaluate(x) -> log_px.data                      models.py:37-40
log_prob(x) == evaluate(x)   (the north-star name; NormalizingFlow is an alias)

The layer loop enqueues one kernel chain per layer on the current HIP stream,
accumulating log|det| in place (no per-layer temporaries, no host syncs); the
reference's errors are raised after the chain from the kernels' status words
(config.STRICT_CHECKS).  An isotropic-normal prior (the reference's "Normal"
prior, applications/src/setup.py:25-30) is evaluated by the fused
nfk_normal_logprob epilogue; any other prior object is called as is.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import config
from . import kernels as K_
from .flows import NSF_CL, RealNVP, _HipFlow, _check_input, _invalidate_after_load, _needs_grad, check_status
from .flows import rnvp_pad, rnvp_unpad

__all__ = ["NormalizingFlowModel", "NormalizingFlow"]


def _iso_normal(prior):
    """(scale, half_log_det) if ``prior`` is MultivariateNormal(0, s^2 I), else None."""
    if not isinstance(prior, torch.distributions.MultivariateNormal):
        return None
    loc = prior.loc
    L = prior.scale_tril
    if loc.dim() != 1 or L.dim() != 2 or L.dtype != torch.float32:
        return None
    d = L.diagonal()
    off = L - torch.diag_embed(d)
    ok = bool((loc == 0).all()) and bool((off == 0).all()) and bool((d == d[0]).all())
    if not ok:
        return None
    hld = float(d.log().sum())  # MultivariateNormal's half_log_det, as torch evaluates it
    return float(d[0]), hld


class _NormalLogProbFn(torch.autograd.Function):
    """log N(z; 0, s^2 I) by the nfk_normal_logprob kernel, differentiable in
    z: d/dz = -z / s^2 (the values are those of the inference path)."""

    @staticmethod
    def forward(ctx, z, scale, hld, status):
        out = torch.empty(z.shape[0], dtype=torch.float32, device=z.device)
        K_.normal_logprob(z, out, scale=scale, hld=hld, status=status)
        ctx.save_for_backward(z)
        ctx.inv_var = 1.0 / (scale * scale)
        return out

    @staticmethod
    def backward(ctx, g):
        z, = ctx.saved_tensors
        return g[:, None] * z * (-ctx.inv_var), None, None, None


def _compose_maps(run, D, device):
    """nfk_fused_nsf_chain's cmaps for a run of NSF_CL layers (include/nfk.h):
    the chain keeps x's column order in its LDS tile and every layer overwrites
    its upper columns in place, so output column o of a layer is the tile
    column its input lo_in[i] / up_in[j] came from (flows.py:239's masked-first
    concatenation).  perm[c] = tile column of the current logical column c."""
    perm = list(range(D))
    out = []
    for flow in run:
        lo_in, lo_out, up_in, up_out = flow._maps(device).lists
        t_lo = [perm[c] for c in lo_in]
        t_up = [perm[c] for c in up_in]
        out += t_lo + t_up
        nxt = [0] * D
        for o, t in zip(lo_out, t_lo):
            nxt[o] = t
        for o, t in zip(up_out, t_up):
            nxt[o] = t
        perm = nxt
    return torch.tensor(out + perm, dtype=torch.int32, device=device)


def _save_maps(run, D, device):
    """nfk_fused_nsf_chain_saved's smaps: for layers 1 .. len(run) - 1 of the
    run, the tile column of each of the layer's input columns (the
    permutation _compose_maps has composed at the start of that layer)."""
    perm = list(range(D))
    out = []
    for i, flow in enumerate(run):
        if i > 0:
            out += perm
        lo_in, lo_out, up_in, up_out = flow._maps(device).lists
        nxt = [0] * D
        for o, c in zip(lo_out, lo_in):
            nxt[o] = perm[c]
        for o, c in zip(up_out, up_in):
            nxt[o] = perm[c]
        perm = nxt
    return torch.tensor(out, dtype=torch.int32, device=device)


class _ChainFn(torch.autograd.Function):
    """A run of fused NSF_CL layers as ONE autograd node (training forward,
    config.USE_TRAIN_CHAIN): the forward is one nfk_fused_nsf_chain_saved
    launch (z, the summed log|det| and every layer's input), the backward
    walks the layers last to first through each layer's own VJP
    (NSF_CL._vjp, as flows._LayerFn calls it) on the saved inputs, so values
    and gradients are bitwise those of one _LayerFn node per layer.

    forward(model, run, shape, status, names, x, *params) -> (z, logdet)
    params: the layers' parameters in order, names[l] those of layer l."""

    @staticmethod
    def forward(ctx, model, run, shape, status, names, x, *params):
        n_lo, n_up, hidden, K, B = shape
        D = n_lo + n_up
        wp, cm = model._chain_args(list(run), D, False, x)
        sm = model._chain_save_maps(run, D, x.device)
        nb = x.shape[0]
        z = torch.empty_like(x, memory_format=torch.contiguous_format)
        ld = torch.empty(nb, dtype=torch.float32, device=x.device)
        saves = torch.empty(len(run) - 1, nb, D, dtype=x.dtype, device=x.device)
        K_.fused_nsf_chain_saved(x, wp, cm, sm, len(run), n_lo, n_up, hidden, z, saves, logdet=ld,
                                 logdet_mode=K_.MODE_WRITE, K=K, tail_bound=B, status=status)
        ctx.run, ctx.names = run, names
        ctx.save_for_backward(x, saves, *params)
        return z, ld

    @staticmethod
    def backward(ctx, gz, gld):
        x, saves, *params = ctx.saved_tensors
        run, names = ctx.run, ctx.names
        need_x = ctx.needs_input_grad[5]
        need_p = ctx.needs_input_grad[6:]
        offs = [0]
        for nm in names:
            offs.append(offs[-1] + len(nm))
        grads = [None] * len(params)
        g = gz
        for l in range(len(run) - 1, -1, -1):
            a, b = offs[l], offs[l + 1]
            need = (l > 0 or need_x,) + tuple(need_p[a:b])
            res = run[l]._vjp(x if l == 0 else saves[l - 1], names[l], params[a:b], g, gld, False, need)
            g = res[0]
            grads[a:b] = res[1:]
        return (None, None, None, None, None, g if need_x else None, *grads)


class NormalizingFlowModel(nn.Module):

    def __init__(self, prior, flows, device="cpu"):
        super().__init__()
        self.device = device
        self.prior = prior
        self.flows = nn.ModuleList(flows)
        self._prior_key = None
        self._prior_iso = None
        self._chain_cache = {}
        self._lp_plan_cache = None
        self.register_load_state_dict_post_hook(_invalidate_after_load)

    def __getstate__(self):
        """Copies and pickles carry no derived state: the chained-launch
        arguments (device pointer tables, and the weight-stream chain's ctypes
        pointer arrays, which neither copy nor pickle) and the log_prob plan are
        rebuilt on the copy's first call, like the layers' packs
        (flows._HipFlow.__getstate__)."""
        state = super().__getstate__()
        state["_chain_cache"] = {}
        state["_lp_plan_cache"] = None
        state["_prior_key"] = None
        state["_prior_iso"] = None
        return state

    def invalidate_caches(self):
        """Drop every cached derivative of the parameters and the prior: the
        layers' fused weight packs, the chained-launch arguments and the
        one-launch log_prob plan.  Needed only after writes the version
        counters cannot see (``p.data.copy_(...)``, ``p.data -= lr * g``, EMA
        updates through ``.data``); optimizer steps and load_state_dict are
        tracked automatically."""
        for f in self.flows:
            if isinstance(f, _HipFlow):
                f.invalidate_caches()
        self._chain_cache = {}
        self._lp_plan_cache = None
        self._prior_key = None
        self._prior_iso = None

    # ------------------------------------------------------------------ prior
    def _prior_consts(self):
        p = self.prior
        key = (id(p),) + tuple((t.data_ptr(), t._version) for t in (p.loc, p.scale_tril)) \
            if isinstance(p, torch.distributions.MultivariateNormal) else (id(p),)
        if key != self._prior_key:
            self._prior_iso = _iso_normal(p)
            self._prior_key = key
        return self._prior_iso

    def _prior_log_prob(self, z, logdet=None, sign=1, status=None):
        """log prior(z) (+ sign * logdet).  The kernel path ORs NFK_ST_NAN_Z into
        ``status`` (one int32 word) on a NaN z, which the caller's status check
        turns into the ValueError of torch's argument validation; any other
        prior is called as is and validates by itself."""
        iso = self._prior_consts()
        if iso is not None and z.shape[1] == self.prior.loc.shape[0]:
            if not (torch.is_grad_enabled() and z.requires_grad):
                out = torch.empty(z.shape[0], dtype=torch.float32, device=z.device)
                K_.normal_logprob(z, out, scale=iso[0], hld=iso[1], logdet=logdet, sign=sign,
                                  status=status)
                return out
            if not (self.prior.loc.requires_grad or self.prior.scale_tril.requires_grad):
                lp = _NormalLogProbFn.apply(z, iso[0], iso[1], status)
                return lp if logdet is None else (lp + logdet if sign >= 0 else lp - logdet)
        lp = self.prior.log_prob(z)
        if logdet is None:
            return lp
        return lp + logdet if sign >= 0 else lp - logdet

    # ------------------------------------------------------------------ chain
    def _status(self, device):
        """One status word per spline-layer slot, plus one for the prior (last)."""
        n = sum(f._n_status for f in self.flows if isinstance(f, _HipFlow))
        return torch.zeros(n + 1, dtype=torch.int32, device=device), n

    def _chain(self, x, inverse, deferred=None):
        """Run the layer chain.  With ``deferred`` (a list) the status check is
        left to the caller, who appends its prior kernel first so the GPU queue
        runs layers + prior back to back before the one host sync.

        Inference accumulates log|det| in place; when autograd needs gradients
        every kernel-backed layer runs as an autograd node (flows._LayerFn) and
        the per-layer log|det| are summed out of place."""
        x = _check_input(x)
        m = x.shape[0]
        grad = _needs_grad(self, x)
        logdet = torch.zeros(m, dtype=torch.float32, device=x.device)
        status, n_st = self._status(x.device)
        off = 0
        flows = self.flows[::-1] if inverse else self.flows
        with torch.set_grad_enabled(grad):
            for item in self._groups(flows, x.device, grad, inverse, batch=m):
                if isinstance(item, tuple):  # a run of fused NSF_CL or RealNVP layers: one launch
                    run, shape = item
                    k = sum(f._n_status for f in run)
                    if grad:
                        x, ld = self._train_chain(run, shape, x, status[off:off + k])
                        logdet = logdet + ld
                    else:
                        x = self._run_chain(run, shape, x, inverse, logdet, status[off:off + k])
                    off += k
                    continue
                flow = item
                if isinstance(flow, _HipFlow):
                    k = flow._n_status
                    st = status[off:off + k] if k else None
                    off += k
                    if grad:
                        x, ld = flow._call(x, inverse, status=st)
                        logdet = logdet + ld
                    else:
                        x = flow._run(x, inverse, logdet, K_.MODE_ACC, st)
                else:  # a user-defined layer: reference protocol
                    x, ld = flow.inverse(x) if inverse else flow.forward(x)
                    logdet = logdet + ld if grad else logdet.add_(ld)
        if deferred is not None:
            deferred.append((status, n_st))
        elif n_st:
            check_status(status, n_st)
        return x, logdet

    @staticmethod
    def _prior_word(deferred):
        status, n_st = deferred[-1]
        return status[n_st:n_st + 1]

    # ------------------------------------------------------- chained launches
    @staticmethod
    def _is_rnvp(shape):
        return shape[0] == "rnvp"

    @staticmethod
    def _is_wide(shape):
        return shape[0] == "wide"

    def _groups(self, flows, device, grad, inverse=False, batch=None):
        """The layer sequence with every run of consecutive NSF_CL layers (or of
        RealNVP layers) that share one fused-kernel shape replaced by (run,
        shape) tuples of at most nfk_fused_nsf_chain_max /
        nfk_fused_realnvp_chain_max layers (runs of one stay single).
        RealNVP shapes are ("rnvp", kernel half_dim, hidden, half_dim): a
        half-dimension the kernel does not take runs zero-padded to one it
        does (RealNVP._fused_half).  Under autograd (``grad``) only NSF_CL runs
        in the forward direction that nfk_fused_nsf_chain_saved takes are
        grouped (config.USE_TRAIN_CHAIN; _ChainFn).  With ``batch``, runs of
        RealNVP layers that take the weight-stream form at that batch
        (RealNVP._wide_pack: Polymer_rnvp's width) group as ("wide", half,
        hidden): one nfk_wide_rnvp_chain call."""
        if not (config.USE_FUSED and config.USE_CHAIN):
            return list(flows)
        if grad and (inverse or not config.USE_TRAIN_CHAIN):
            return list(flows)
        out, run, shape = [], [], None

        def flush():
            if shape is None:
                nmax = 0
            elif self._is_wide(shape):
                nmax = len(run)
            elif self._is_rnvp(shape):
                nmax = K_.fused_realnvp_chain_max(shape[1], shape[2])
            else:
                nmax = K_.fused_nsf_chain_max(*shape[:4])
                if grad:  # the saved form also holds the save maps: its limit can be lower
                    while nmax > 1 and not K_.fused_nsf_chain_saved_ok(*shape[:4], nmax):
                        nmax -= 1
            i = 0
            while i < len(run):
                piece = run[i:i + max(nmax, 1)]
                if len(piece) > 1 and (not grad or K_.fused_nsf_chain_saved_ok(*shape[:4], len(piece))):
                    out.append((piece, shape))
                else:
                    out.extend(piece)
                i += len(piece)

        kinds = (NSF_CL,) if grad else (NSF_CL, RealNVP)
        for flow in flows:
            sh = flow._chain_shape(device) if isinstance(flow, kinds) else None
            if sh is None and batch is not None and not grad and isinstance(flow, RealNVP):
                wp = flow._wide_pack(device, batch)
                sh = ("wide", wp.half, wp.hidden) if wp is not None else None
            if sh is not None and sh == shape:
                run.append(flow)
                continue
            flush()
            run, shape = ([flow], sh) if sh is not None else ([], None)
            if sh is None:
                out.append(flow)
        flush()
        return out

    @staticmethod
    def _chain_layout_ok(x, D):
        return x.shape[1] == D and x.data_ptr() % 16 == 0 and x.stride(1) == 1 and x.stride(0) % 4 == 0

    def _chain_args(self, run, D, inverse, x):
        packs = [f._fused_pack(x.device) for f in run]
        key = (tuple(id(f) for f in run), bool(inverse), str(x.device))
        ent = self._chain_cache.get(key)
        ptrs = tuple(p.data_ptr() for p in packs)
        if ent is None or ent[0] != ptrs:
            maps = None if isinstance(run[0], RealNVP) else _compose_maps(run, D, x.device)
            ent = (ptrs, torch.tensor(ptrs, dtype=torch.int64, device=x.device), maps)
            self._chain_cache[key] = ent
        return ent[1], ent[2]

    def _chain_save_maps(self, run, D, device):
        key = ("save", tuple(id(f) for f in run), str(device))
        sm = self._chain_cache.get(key)
        if sm is None:
            sm = self._chain_cache[key] = _save_maps(run, D, device)
        return sm

    def _train_chain(self, run, shape, x, status):
        """A run of fused NSF_CL layers under autograd: one _ChainFn node."""
        D = shape[0] + shape[1]
        if x.dim() != 2 or x.shape[1] != D:
            # not the run's width: per-layer nodes, whose first layer raises the
            # reference's error (the chain kernel would read past or truncate x)
            logdet = torch.zeros(x.shape[0], dtype=torch.float32, device=x.device)
            for i, flow in enumerate(run):
                x, ld = flow._call(x, False, status=status[i:i + 1] if flow._n_status else None)
                logdet = logdet + ld
            return x, logdet
        if not self._chain_layout_ok(x, D):
            x = x.clone(memory_format=torch.contiguous_format)  # fresh, 16-byte aligned rows
        named = [list(f.named_parameters()) for f in run]
        names = tuple(tuple(n for n, _ in nm) for nm in named)
        return _ChainFn.apply(self, tuple(run), shape, status, names, x, *(t for nm in named for _, t in nm))

    def _fused_log_prob(self, x):
        """evaluate() as ONE launch when the whole model is one chained run of
        fused NSF_CL layers and the prior is the isotropic Normal: the prior
        is the chain's epilogue and z never reaches HBM.  None otherwise."""
        if not (config.USE_FUSED and config.USE_CHAIN) or x.dim() != 2 or not x.is_cuda \
                or x.dtype != torch.float32:
            return None
        # only a model made entirely of NSF_CL (or of RealNVP) layers can be one
        # chained run: skip the plan's parameter key (a walk of every parameter)
        # for any other model
        fl = self.flows
        if len(fl) < 2 or not (all(isinstance(f, NSF_CL) for f in fl) or all(isinstance(f, RealNVP) for f in fl)):
            return None
        plan = self._lp_plan(x)
        if plan is None:
            return None
        run, shape, iso, wp, cm = plan
        out = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
        if self._is_rnvp(shape):
            _, hp, hidden, h = shape
            if x.shape[1] != 2 * h or (hp == h and not self._chain_layout_ok(x, 2 * h)):
                return None  # (a padded copy is laid out for the chain by construction)
            status = torch.zeros(1, dtype=torch.int32, device=x.device)  # the prior's NaN-z word
            # padded halves: z's padded columns are 0, and the kernel's constant
            # 2 hp log(2 pi) is brought back to the true 2 h log(2 pi) through hld
            hld = iso[1] - (hp - h) * math.log(2 * math.pi)
            K_.fused_realnvp_chain(rnvp_pad(x, h, hp), wp, len(run), hp, hidden, None, logdet=None,
                                   logdet_mode=K_.MODE_NONE, inverse=False, status=status, log_prob=out,
                                   prior_scale=iso[0], prior_hld=hld)
            check_status(status, 0, prior=self.prior)
            return out
        n_lo, n_up, hidden, K, B = shape
        if not self._chain_layout_ok(x, n_lo + n_up):
            return None
        status = torch.zeros(len(run), dtype=torch.int32, device=x.device)
        K_.fused_nsf_chain(x, wp, cm, len(run), n_lo, n_up, hidden, None, logdet=None,
                           logdet_mode=K_.MODE_NONE, K=K, tail_bound=B, inverse=False, status=status,
                           log_prob=out, prior_scale=iso[0], prior_hld=iso[1])
        check_status(status, len(run), prior=self.prior)
        return out

    def _lp_plan(self, x):
        """(run, shape, prior consts, wpacks, cmaps) of the one-launch evaluate, or
        None; cached on the parameters' storage and versions so a log_prob loop
        pays one key check per call instead of re-deriving the plan."""
        iso = self._prior_consts()
        # the structure the plan depends on besides the parameters: the layer
        # objects (a parameter-free layer appended changes the run), each spline
        # layer's tail bound, bin count and mask object (part of the chain shape
        # and maps), and the prior's dimension (checked again outside the cache)
        struct = tuple((id(f), getattr(f, "B", None), getattr(f, "K", None), id(getattr(f, "mask", None)))
                       for f in self.flows)
        key = (str(x.device), iso, struct, tuple((p.data_ptr(), p._version) for p in self.parameters()))
        if self._lp_plan_cache is not None and self._lp_plan_cache[0] == key:
            plan = self._lp_plan_cache[1]
        else:
            plan = None
            groups = self._groups(self.flows, x.device, False)
            if iso is not None and len(groups) == 1 and isinstance(groups[0], tuple):
                run, shape = groups[0]
                wp, cm = self._chain_args(run, self._shape_dim(shape), False, x)
                plan = (run, shape, iso, wp, cm)
            self._lp_plan_cache = (key, plan)
        if plan is not None and self.prior.loc.shape[0] != self._shape_dim(plan[1]):
            return None  # the prior's dimension does not match: the generic path raises like torch
        return plan

    @classmethod
    def _shape_dim(cls, shape):
        return 2 * shape[3] if cls._is_rnvp(shape) else shape[0] + shape[1]

    def _run_chain(self, run, shape, x, inverse, logdet, status):
        if self._is_wide(shape):
            # consecutive weight-stream RealNVP layers: one call (the packs were
            # validated by _wide_pack while grouping; the host pointer tables
            # are kept per run and rebuilt when any layer's pack changed)
            wps = tuple(f._wide_pack(x.device, x.shape[0]) for f in run)
            key = ("wide", tuple(id(f) for f in run), str(x.device))
            ent = self._chain_cache.get(key)
            if ent is None or len(ent[0]) != len(wps) or any(a is not b for a, b in zip(ent[0], wps)):
                ent = self._chain_cache[key] = (wps, K_.WideRnvpChain(list(wps)))
            xc = x if x.stride(1) == 1 else x.contiguous()
            z = torch.empty_like(xc, memory_format=torch.contiguous_format)
            K_.wide_rnvp_chain(xc, ent[1], z, logdet=logdet, logdet_mode=K_.MODE_ACC, inverse=inverse)
            return z
        if self._is_rnvp(shape):
            _, hp, hidden, h = shape
            if x.shape[1] != 2 * h or (hp == h and not self._chain_layout_ok(x, 2 * h)):
                for flow in run:  # not the chain's layout: one launch per layer
                    x = flow._run(x, inverse, logdet, K_.MODE_ACC, None)
                return x
            wp, _ = self._chain_args(run, 2 * h, inverse, x)
            xk = rnvp_pad(x, h, hp)
            z = torch.empty_like(xk, memory_format=torch.contiguous_format)
            K_.fused_realnvp_chain(xk, wp, len(run), hp, hidden, z, logdet=logdet, logdet_mode=K_.MODE_ACC,
                                   inverse=inverse)
            return rnvp_unpad(z, h, hp)
        n_lo, n_up, hidden, K, B = shape
        D = n_lo + n_up
        if not self._chain_layout_ok(x, D):
            for flow in run:  # not the chain's layout: one launch per layer
                x = flow._run(x, inverse, logdet, K_.MODE_ACC, status[:1])
                status = status[1:]
            return x
        wp, cm = self._chain_args(run, D, inverse, x)
        z = torch.empty_like(x, memory_format=torch.contiguous_format)
        K_.fused_nsf_chain(x, wp, cm, len(run), n_lo, n_up, hidden, z, logdet=logdet,
                           logdet_mode=K_.MODE_ACC, K=K, tail_bound=B, inverse=inverse, status=status)
        return z

    def _check(self, deferred, prior=False):
        """The deferred status check of a chain (+ its prior word when
        ``prior``: the NaN-z ValueError of the prior's argument validation)."""
        for status, n_st in deferred:
            if n_st or prior:
                check_status(status, n_st, prior=self.prior if prior else None)

    # ------------------------------------------------------------------ API
    def forward(self, x):
        d = []
        z, log_det = self._chain(x, False, d)
        lp = self._prior_log_prob(z, status=self._prior_word(d))
        self._check(d, prior=True)
        return z, lp, log_det

    def inverse(self, z):
        return self._chain(z, True)

    # sample / evaluate return detached ``.data`` (models.py:35, 40), so they
    # never build a graph: the in-place kernel chain serves them even in grad mode
    @torch.no_grad()
    def sample(self, n_samples):
        z = self.prior.sample((n_samples,))
        d = []
        x, log_det = self._chain(z, True, d)
        log_px = self._prior_log_prob(z, logdet=log_det, sign=-1, status=self._prior_word(d))
        self._check(d, prior=True)
        return x.data, log_px.data, z.data

    @torch.no_grad()
    def evaluate(self, x):
        out = self._fused_log_prob(x)
        if out is not None:
            return out.data
        d = []
        z, log_det = self._chain(x, False, d)
        out = self._prior_log_prob(z, logdet=log_det, sign=1, status=self._prior_word(d))
        self._check(d, prior=True)
        return out.data

    def log_prob(self, x):
        return self.evaluate(x)


NormalizingFlow = NormalizingFlowModel
