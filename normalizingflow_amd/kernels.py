"""Validated Python wrappers over the libnfk.so entry points.

Each wrapper checks device / dtype / layout on the host (no device sync),
then enqueues the kernel on the tensor's current HIP stream.  They are the
only place the package touches raw pointers.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib, config

F32 = torch.float32

MODE_NONE, MODE_WRITE, MODE_ACC = 0, 1, 2


class KernelTimer:
    """Optional per-entry-point timing with HIP events recorded on the stream
    each kernel is enqueued on (torch's current stream).  Install with
    ``kernels.TIMER = KernelTimer()``; read ``summary()`` after a sync."""

    def __init__(self):
        self.events = {}

    def start(self, name, dev):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(dev))
        return ev

    def stop(self, name, dev, ev0):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(dev))
        self.events.setdefault(name, []).append((ev0, ev))

    def summary(self):
        """name -> (launches, mean ms, total ms)"""
        out = {}
        for name, evs in self.events.items():
            ms = [a.elapsed_time(b) for a, b in evs]
            out[name] = (len(ms), sum(ms) / len(ms), sum(ms))
        return out


TIMER = None


def _timed(name, dev, fn, *args):
    if TIMER is None:
        return _lib.call(fn, *args)
    ev0 = TIMER.start(name, dev)
    rc = _lib.call(fn, *args)
    TIMER.stop(name, dev, ev0)
    return rc


def _require_hip(*ts):
    dev = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(
                "normalizingflow_amd runs on the ROCm device only (tensor on %s); move the model "
                "and inputs to 'cuda' -- there is no CPU fallback" % t.device)
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError("tensors on different devices: %s vs %s" % (dev, t.device))
    return dev


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def _ptr(t):
    return None if t is None else t.data_ptr()


def _mat(t, name):
    """(ptr, row stride) of a 2-D fp32 tensor with unit column stride."""
    if t.dtype != F32:
        raise TypeError("%s must be float32, got %s" % (name, t.dtype))
    if t.dim() != 2:
        raise ValueError("%s must be 2-D, got shape %s" % (name, tuple(t.shape)))
    if t.shape[1] > 1 and t.stride(1) != 1:
        raise ValueError("%s needs unit column stride" % name)
    return t.data_ptr(), (t.stride(0) if t.shape[0] > 1 else max(t.shape[1], 1))


def _vec(t, n, name, dtype=F32):
    if t is None:
        return None
    if t.dtype != dtype or t.numel() != n or (n > 1 and not t.is_contiguous()):
        raise ValueError("%s must be a contiguous %s vector of %d elements" % (name, dtype, n))
    return t.data_ptr()


# ---------------------------------------------------------------------------
def rqs_coupling(x, params, up_in, up_out, z, *, lo_in=None, lo_out=None, logdet=None,
                 logdet_mode=MODE_NONE, lad_out=None, K, left, right, bottom, top, tails=True,
                 min_bin_width=1e-3, min_bin_height=1e-3, min_derivative=1e-3, param_mode=0,
                 inverse=False, status=None):
    """Spline coupling (nfk_rqs_coupling).  params: dense [B, n_up*(3K-1)] (or 3-D)."""
    dev = _require_hip(x, params, up_in, z, logdet, lad_out, status)
    B = x.shape[0]
    n_up = up_in.numel()
    n_lo = 0 if lo_in is None else lo_in.numel()
    per = 3 * K + 1 if param_mode == 2 else 3 * K - 1
    if params.dtype != F32 or not params.is_contiguous() or params.numel() != B * n_up * per:
        raise ValueError("params must be a dense float32 [B, n_up, %d] tensor "
                         "(got %s, %s)" % (per, tuple(params.shape), params.dtype))
    xp, ldx = _mat(x, "x")
    zp, ldz = _mat(z, "z")
    if z.shape[0] != B:
        raise ValueError("z batch mismatch")
    lp, ldl = (None, 0) if lad_out is None else _mat(lad_out, "lad_out")
    for m in (up_in, up_out, lo_in, lo_out):
        if m is not None and (m.dtype != torch.int32 or not m.is_contiguous()):
            raise ValueError("index maps must be contiguous int32")
    _timed("nfk_rqs_coupling", dev, "nfk_rqs_coupling", xp, ldx, params.data_ptr(), up_in.data_ptr(),
              up_out.data_ptr(), n_up, _ptr(lo_in), _ptr(lo_out), n_lo, zp, ldz,
              _vec(logdet, B, "logdet"), logdet_mode, lp, ldl, B, K, float(left), float(right),
              float(bottom), float(top), 1 if tails else 0, float(min_bin_width),
              float(min_bin_height), float(min_derivative), param_mode, 1 if inverse else 0,
              _vec(status, 1, "status", torch.int32), _stream(dev))


def rqs_coupling_bwd(x, params, up_in, up_out, gz, glogdet, gparams, gx, *, lo_in=None,
                     lo_out=None, K, left, right, bottom, top, tails=True, min_bin_width=1e-3,
                     min_bin_height=1e-3, min_derivative=1e-3, param_mode=0, inverse=False):
    """Backward of rqs_coupling (nfk_rqs_coupling_bwd): writes gparams (layout of
    params) and gx (upper columns = dL/dx, lower columns = gz pass-through)."""
    dev = _require_hip(x, params, up_in, gz, glogdet, gparams, gx)
    B = x.shape[0]
    n_up = up_in.numel()
    n_lo = 0 if lo_in is None else lo_in.numel()
    per = 3 * K + 1 if param_mode == 2 else 3 * K - 1
    for name, t in (("params", params), ("gparams", gparams)):
        if t.dtype != F32 or not t.is_contiguous() or t.numel() != B * n_up * per:
            raise ValueError("%s must be a dense float32 [B, n_up, %d] tensor" % (name, per))
    xp, ldx = _mat(x, "x")
    gxp, ldgx = _mat(gx, "gx")
    gzp, ldgz = (None, 0) if gz is None else _mat(gz, "gz")
    if gx.shape[0] != B or (gz is not None and gz.shape[0] != B):
        raise ValueError("gradient batch mismatch")
    for m in (up_in, up_out, lo_in, lo_out):
        if m is not None and (m.dtype != torch.int32 or not m.is_contiguous()):
            raise ValueError("index maps must be contiguous int32")
    _timed("nfk_rqs_coupling_bwd", dev, "nfk_rqs_coupling_bwd", xp, ldx, params.data_ptr(),
           up_in.data_ptr(), up_out.data_ptr(), n_up, _ptr(lo_in), _ptr(lo_out), n_lo, gzp, ldgz,
           _vec(glogdet, B, "glogdet"), gparams.data_ptr(), gxp, ldgx, B, K, float(left),
           float(right), float(bottom), float(top), 1 if tails else 0, float(min_bin_width),
           float(min_bin_height), float(min_derivative), param_mode, 1 if inverse else 0,
           _stream(dev))


def maf(x, init_param, params, out, c0, c1, *, logdet=None, logdet_mode=MODE_NONE,
        inverse=False):
    """MAF per-coordinate affine map of columns [c0, c1) (nfk_maf)."""
    dev = _require_hip(x, init_param, params, out, logdet)
    B, dim = x.shape
    if out.shape != x.shape:
        raise ValueError("out must match x")
    if init_param.dtype != F32 or init_param.numel() != 2 or not init_param.is_contiguous():
        raise ValueError("init_param must be a contiguous float32 [2] tensor")
    pp, ldp = (None, 0)
    if params is not None:
        pp, ldp = _mat(params, "params")
        if params.shape[0] != B or params.shape[1] < 2 * (c1 - max(c0, 1)):
            raise ValueError("params must be [B, >= 2 x columns]")
    elif c1 > 1:
        raise ValueError("params are required for columns >= 1")
    xp, ldx = _mat(x, "x")
    op, ldo = _mat(out, "out")
    _lib.call("nfk_maf", xp, ldx, init_param.data_ptr(), pp, ldp, int(c0), int(c1), dim, op, ldo,
              _vec(logdet, B, "logdet"), logdet_mode, B, 1 if inverse else 0, _stream(dev))


def actnorm(x, mu, log_sigma, z, *, logdet=None, logdet_mode=MODE_NONE, ld_scalar=None,
            inverse=False):
    """ActNorm (nfk_actnorm)."""
    dev = _require_hip(x, mu, log_sigma, z, logdet, ld_scalar)
    B, dim = x.shape
    for name, t in (("mu", mu), ("log_sigma", log_sigma)):
        if t.dtype != F32 or t.numel() != dim or not t.is_contiguous():
            raise ValueError("%s must be a contiguous float32 [%d] tensor" % (name, dim))
    xp, ldx = _mat(x, "x")
    zp, ldz = _mat(z, "z")
    _lib.call("nfk_actnorm", xp, ldx, mu.data_ptr(), log_sigma.data_ptr(), dim, zp, ldz,
              _vec(logdet, B, "logdet"), logdet_mode, _vec(ld_scalar, 1, "ld_scalar"), B,
              1 if inverse else 0, _stream(dev))


def searchsorted(bin_locations, inputs, eps=1e-6):
    dev = _require_hip(bin_locations, inputs)
    if bin_locations.dtype != F32 or not bin_locations.is_contiguous():
        raise ValueError("bin_locations must be contiguous float32")
    n = bin_locations.shape[-1]
    rows = bin_locations.numel() // n
    if inputs.numel() != rows:
        raise ValueError("inputs must have one value per bin row")
    v = inputs.contiguous().to(F32)
    idx = torch.empty(inputs.shape, dtype=torch.int64, device=dev)
    _lib.call("nfk_searchsorted", bin_locations.data_ptr(), v.data_ptr(), idx.data_ptr(), rows,
              n, float(eps), _stream(dev))
    return idx


def affine_coupling(x_in, s, t, x_out, *, logdet=None, logdet_mode=MODE_NONE, inverse=False):
    dev = _require_hip(x_in, s, t, x_out, logdet)
    B, n = x_in.shape
    if s.shape != (B, n) or t.shape != (B, n) or x_out.shape != (B, n):
        raise ValueError("affine coupling shape mismatch: in %s s %s t %s out %s"
                         % (tuple(x_in.shape), tuple(s.shape), tuple(t.shape), tuple(x_out.shape)))
    xp, ldi = _mat(x_in, "x_in")
    sp, lds = _mat(s, "s")
    tp, ldt = _mat(t, "t")
    if ldt != lds:
        if B > 1:
            t = t.contiguous() if t.stride(0) != lds else t
            s = s.contiguous()
            sp, lds = _mat(s, "s")
            tp, ldt = _mat(t, "t")
        ldt = lds
    op, ldo = _mat(x_out, "x_out")
    _timed("nfk_affine_coupling", dev, "nfk_affine_coupling", xp, ldi, sp, tp, lds, op, ldo, _vec(logdet, B, "logdet"),
              logdet_mode, B, n, 1 if inverse else 0, _stream(dev))


def affine_coupling_bwd(x_in, s, t, g_out, g_logdet, g_in, g_s, g_t=None, *, accumulate=False, inverse=False):
    """VJP of affine_coupling (include/nfk.h nfk_affine_coupling_bwd); g_s / g_t
    are written (contiguous [B, n]), g_in written or accumulated."""
    dev = _require_hip(x_in, s, t, g_out, g_logdet, g_in, g_s, g_t)
    B, n = x_in.shape
    for name, v in (("s", s), ("t", t), ("g_out", g_out), ("g_in", g_in), ("g_s", g_s), ("g_t", g_t)):
        if v is not None and tuple(v.shape) != (B, n):
            raise ValueError("affine_coupling_bwd: %s has shape %s, want %s" % (name, tuple(v.shape), (B, n)))
    if inverse and (t is None or g_t is None):
        raise ValueError("affine_coupling_bwd: the inverse needs t and g_t")
    xp, ldi = _mat(x_in, "x_in")
    sp, lds = _mat(s, "s")
    tp = None
    if t is not None:
        tp, ldt = _mat(t, "t")
        if ldt != lds and B > 1:
            raise ValueError("affine_coupling_bwd: s and t need one row stride")
    gp, ldg = _mat(g_out, "g_out") if g_out is not None else (None, 0)
    ip, ldgi = _mat(g_in, "g_in")
    gsp, ldgs = _mat(g_s, "g_s")
    gtp = None
    if g_t is not None:
        gtp, ldgt = _mat(g_t, "g_t")
        if ldgt != ldgs and B > 1:
            raise ValueError("affine_coupling_bwd: g_s and g_t need one row stride")
    _timed("nfk_affine_coupling_bwd", dev, "nfk_affine_coupling_bwd", xp, ldi, sp, tp, lds, gp, ldg,
           _vec(g_logdet, B, "g_logdet"), ip, ldgi, 1 if accumulate else 0, gsp, gtp, ldgs, B, n,
           1 if inverse else 0, _stream(dev))


PLANAR_NL = {"tanh": 0, "leaky_relu": 1, "elu": 2}


def planar(x, w, u, b, z, *, logdet=None, logdet_mode=MODE_NONE, ld_out=None, nonlinearity=0):
    dev = _require_hip(x, w, u, b, z, logdet, ld_out)
    B, D = x.shape
    xp, ldx = _mat(x, "x")
    zp, ldz = _mat(z, "z")
    _lib.call("nfk_planar", xp, ldx, _vec(w, D, "w"), _vec(u, D, "u"), _vec(b, 1, "b"), zp, ldz,
              _vec(logdet, B, "logdet"), logdet_mode, _vec(ld_out, B, "ld_out"), B, D,
              nonlinearity, _stream(dev))


def radial_workspace_elems():
    return int(_lib.load().nfk_radial_workspace_elems())


def radial_sumsq(x, x0, workspace, sumsq):
    dev = _require_hip(x, x0, workspace, sumsq)
    B, D = x.shape
    xp, ldx = _mat(x, "x")
    _lib.call("nfk_radial_sumsq", xp, ldx, _vec(x0, D, "x0"),
              B, D, _vec(workspace, radial_workspace_elems(), "workspace", torch.float64),
              _vec(sumsq, 1, "sumsq", torch.float64), _stream(dev))


def radial_apply(x, x0, log_alpha, beta, sumsq, z, ld_scalar, *, logdet=None,
                 logdet_mode=MODE_NONE):
    dev = _require_hip(x, x0, log_alpha, beta, sumsq, z, ld_scalar, logdet)
    B, D = x.shape
    xp, ldx = _mat(x, "x")
    zp, ldz = _mat(z, "z")
    _lib.call("nfk_radial_apply", xp, ldx, _vec(x0, D, "x0"), _vec(log_alpha, 1, "log_alpha"),
              _vec(beta, 1, "beta"), _vec(sumsq, 1, "sumsq", torch.float64), zp, ldz,
              _vec(ld_scalar, 1, "ld_scalar"), _vec(logdet, B, "logdet"), logdet_mode, B, D,
              _stream(dev))


# ---- FCNN backward input-gradient GEMMs (nfk_fcnn_bwd.hip)
def fcnn_dh_pack_floats(P, H):
    return int(_lib.load().nfk_fcnn_dh_pack_floats(int(P), int(H)))


def fcnn_dh_pack(W):
    """Pack an nn.Linear weight W [P, H] for fcnn_dh (None: shape unsupported)."""
    P, H = W.shape
    n = fcnn_dh_pack_floats(P, H)
    if n == 0:
        return None
    dev = _require_hip(W)
    Wc = W.detach().to(F32).contiguous()
    pack = torch.empty(n, dtype=F32, device=W.device)
    _lib.call("nfk_fcnn_dh_pack", Wc.data_ptr(), P, H, pack.data_ptr(), _stream(dev))
    return pack


def fcnn_dh(g, pack, W_shape, h, out, *, accumulate=False):
    """out (+)= (g @ W) * (1 - h^2) (h None: g @ W), W packed by fcnn_dh_pack;
    out may be a column-strided view (e.g. x's lower columns)."""
    dev = _require_hip(g, pack, h, out)
    P, H = W_shape
    B = g.shape[0]
    gp_, ldg = _mat(g, "g")
    if g.shape[1] != P or tuple(out.shape) != (B, H) or (h is not None and h.shape != (B, H)):
        raise ValueError("fcnn_dh: shape mismatch")
    if out.dtype != F32 or out.dim() != 2:
        raise ValueError("fcnn_dh: out must be a 2-D float32 tensor")
    hp, ldh = _mat(h, "h") if h is not None else (None, 0)
    ldo = out.stride(0) if B > 1 else H * max(out.stride(1), 1)
    cso = out.stride(1) if H > 1 else 1
    _timed("nfk_fcnn_dh", dev, "nfk_fcnn_dh", gp_, ldg, P, pack.data_ptr(), hp, ldh, H, out.data_ptr(), ldo,
           cso, 1 if accumulate else 0, B, _stream(dev))


def gather_cols_ones(x, cols):
    """[x[:, cols] | 1] as the first n + 1 columns of a [B, ceil4(n + 1)]
    buffer (include/nfk.h nfk_gather_cols_ones); returns that [B, n + 1] view."""
    dev = _require_hip(x, cols)
    xp, ldx = _mat(x, "x")
    B, n = x.shape[0], cols.numel()
    ldo = (n + 4) // 4 * 4
    out = torch.empty(B, ldo, dtype=F32, device=dev)
    _lib.call("nfk_gather_cols_ones", xp, ldx, cols.data_ptr(), n, B, out.data_ptr(), ldo, _stream(dev))
    return out[:, :n + 1]


def fcnn_linear(x, pack, W_shape, bias, out, *, tanh=False):
    """out = x @ W + bias (tanh'd when ``tanh``), W [P, H] packed by fcnn_dh_pack
    (an nn.Linear's weight transposed): the FCNN forward on the same kernel."""
    dev = _require_hip(x, pack, bias, out)
    P, H = W_shape
    B = x.shape[0]
    xp, ldx = _mat(x, "x")
    op, ldo = _mat(out, "out")
    if x.shape[1] != P or tuple(out.shape) != (B, H):
        raise ValueError("fcnn_linear: shape mismatch")
    _timed("nfk_fcnn_linear", dev, "nfk_fcnn_linear", xp, ldx, P, pack.data_ptr(), _vec(bias, H, "bias"),
           1 if tanh else 0, H, op, ldo, B, _stream(dev))


# ---- training backward of the remaining flow classes (nfk_flows_bwd.hip)
def flows_bwd_workspace(batch, dim, device):
    """Scratch of nfk_flows_bwd_workspace_bytes (uint8, 256-byte aligned by the allocator)."""
    n = int(_lib.load().nfk_flows_bwd_workspace_bytes(int(batch), int(max(dim, 2))))
    return torch.empty(n, dtype=torch.uint8, device=device)


def planar_bwd(x, w, u, b, gz, glogdet, gx, gw, gu, gb, *, nonlinearity=0):
    """VJP of planar (nfk_planar_bwd): gx [B, D] and the parameter gradients."""
    dev = _require_hip(x, w, u, b, gz, glogdet, gx, gw, gu, gb)
    B, D = x.shape
    xp, ldx = _mat(x, "x")
    gp, ldg = _mat(gz, "gz") if gz is not None else (None, 0)
    gxp, ldgx = _mat(gx, "gx")
    ws = flows_bwd_workspace(B, D, x.device)
    _timed("nfk_planar_bwd", dev, "nfk_planar_bwd", xp, ldx, _vec(w, D, "w"), _vec(u, D, "u"), _vec(b, 1, "b"),
           gp, ldg, _vec(glogdet, B, "glogdet"), gxp, ldgx, _vec(gw, D, "gw"), _vec(gu, D, "gu"),
           _vec(gb, 1, "gb"), ws.data_ptr(), B, D, int(nonlinearity), _stream(dev))


def actnorm_bwd(x, mu, log_sigma, gz, gld, gx, gmu, gls, *, inverse=False):
    """VJP of actnorm (nfk_actnorm_bwd); gld: the scalar log|det|'s gradient ([1] or None)."""
    dev = _require_hip(x, mu, log_sigma, gz, gld, gx, gmu, gls)
    B, D = x.shape
    xp, ldx = _mat(x, "x")
    gp, ldg = _mat(gz, "gz")
    gxp, ldgx = _mat(gx, "gx")
    ws = flows_bwd_workspace(B, D, x.device)
    _timed("nfk_actnorm_bwd", dev, "nfk_actnorm_bwd", xp, ldx, _vec(mu, D, "mu"), _vec(log_sigma, D, "log_sigma"),
           D, gp, ldg, _vec(gld, 1, "gld"), gxp, ldgx, _vec(gmu, D, "gmu"), _vec(gls, D, "gls"), ws.data_ptr(),
           B, 1 if inverse else 0, _stream(dev))


def radial_bwd_scalars(x, x0, log_alpha, beta, sumsq, gz, gld, scal, workspace):
    """First half of Radial's VJP (nfk_radial_bwd_scalars): scal = [dL/dsumsq,
    dL/dlog_alpha, dL/dbeta, beta_hat h]; all-reduce scal[0] across shards
    before radial_bwd_apply."""
    dev = _require_hip(x, x0, log_alpha, beta, sumsq, gz, gld, scal, workspace)
    B, D = x.shape
    xp, ldx = _mat(x, "x")
    gp, ldg = _mat(gz, "gz") if gz is not None else (None, 0)
    _timed("nfk_radial_bwd_scalars", dev, "nfk_radial_bwd_scalars", xp, ldx, _vec(x0, D, "x0"),
           _vec(log_alpha, 1, "log_alpha"), _vec(beta, 1, "beta"), _vec(sumsq, 1, "sumsq", torch.float64),
           gp, ldg, _vec(gld, 1, "gld"), _vec(scal, 4, "scal"), workspace.data_ptr(), B, D, _stream(dev))


def radial_bwd_apply(x, x0, gz, scal, gx, gx0, workspace):
    dev = _require_hip(x, x0, gz, scal, gx, gx0, workspace)
    B, D = x.shape
    xp, ldx = _mat(x, "x")
    gp, ldg = _mat(gz, "gz") if gz is not None else (None, 0)
    gxp, ldgx = _mat(gx, "gx")
    _timed("nfk_radial_bwd_apply", dev, "nfk_radial_bwd_apply", xp, ldx, _vec(x0, D, "x0"), gp, ldg,
           _vec(scal, 4, "scal"), gxp, ldgx, _vec(gx0, D, "gx0"), workspace.data_ptr(), B, D, _stream(dev))


def maf_bwd(x, init_param, params, gout, glogdet, c0, c1, gx, gparams, ginit, *, inverse=False):
    """VJP of maf over columns [c0, c1) (nfk_maf_bwd)."""
    dev = _require_hip(x, init_param, params, gout, glogdet, gx, gparams, ginit)
    B, dim = x.shape
    xp, ldx = _mat(x, "x")
    pp, ldp = _mat(params, "params") if params is not None else (None, 0)
    gpp, ldgp = _mat(gparams, "gparams") if gparams is not None else (None, 0)
    gop, ldgo = _mat(gout, "gout") if gout is not None else (None, 0)
    gxp, ldgx = _mat(gx, "gx")
    ws = flows_bwd_workspace(B, 2, x.device)
    _timed("nfk_maf_bwd", dev, "nfk_maf_bwd", xp, ldx, _vec(init_param, 2, "init_param"), pp, ldp, gop, ldgo,
           _vec(glogdet, B, "glogdet"), int(c0), int(c1), dim, gxp, ldgx, gpp, ldgp, _vec(ginit, 2, "ginit"),
           ws.data_ptr(), B, 1 if inverse else 0, _stream(dev))


def trig_features_bwd(x, gfeat, gx, B):
    """gx[:, :n] += dL/dx through trig_features (nfk_trig_features_bwd)."""
    dev = _require_hip(x, gfeat, gx)
    n_rows, n = x.shape
    xp, ldx = _mat(x, "x")
    fp, ldf = _mat(gfeat, "gfeat")
    gp, ldg = _mat(gx, "gx")
    if gfeat.shape != (n_rows, 2 * n) or gx.shape[0] != n_rows or gx.shape[1] < n:
        raise ValueError("trig_features_bwd: gfeat must be [B, 2n] and gx [B, >=n]")
    _timed("nfk_trig_features_bwd", dev, "nfk_trig_features_bwd", xp, ldx, fp, ldf, gp, ldg, n_rows, n, float(B),
           _stream(dev))


def iso_normal_consts(var, dim):
    """(scale, half_log_det) of MultivariateNormal(0, var*I) as torch evaluates
    them: scale = fp32 Cholesky diagonal, half_log_det = fp32 sum of its logs."""
    cov = torch.eye(dim, dtype=torch.float32) * var
    L = torch.linalg.cholesky(cov)
    return float(L[0, 0]), float(L.diagonal().log().sum())


def normal_logprob(z, out, *, scale=1.0, hld=0.0, logdet=None, sign=1, status=None):
    """``status`` (optional int32 word): NFK_ST_NAN_Z is OR-ed in when z holds a NaN."""
    dev = _require_hip(z, out, logdet, status)
    B, D = z.shape
    zp, ldz = _mat(z, "z")
    _timed("nfk_normal_logprob", dev, "nfk_normal_logprob", zp, ldz, _vec(logdet, B, "logdet"), _vec(out, B, "out"), B, D,
              float(scale), float(hld), int(sign), _vec(status, 1, "status", torch.int32), _stream(dev))


def trig_features(x, feat, B):
    dev = _require_hip(x, feat)
    n_rows, n = x.shape
    xp, ldx = _mat(x, "x")
    fp, ldf = _mat(feat, "feat")
    if feat.shape != (n_rows, 2 * n):
        raise ValueError("feat must be [B, 2n]")
    _lib.call("nfk_trig_features", xp, ldx, fp, ldf, n_rows, n, float(B), _stream(dev))


# ---------------------------------------------------------------------------
def fused_ar_supported(dim, hidden, K):
    return bool(_lib.load().nfk_fused_ar_supported(dim, hidden, K))


def fused_ar_inverse_supported(dim, hidden, K):
    """False for the shapes only the streamed forward covers (their inverse,
    sequential through the outputs, runs per column)."""
    return bool(_lib.load().nfk_fused_ar_inverse_supported(dim, hidden, K))


def fused_ar_pack(weights, init_param, dim, hidden, K):
    """The fused NSF_AR pack from the conditioners' Linear parameters:
    ``weights`` = [(W1, b1, W2, b2, W3, b3) for conditioner 1 .. dim-1].
    Returns (pack, keep): ``keep`` = (device pointer table, init_param, the
    tensors -- contiguous copies where needed, alive until the stream has run
    the pack kernel --, the same pointers as a host array for ar_seqinv)."""
    flat = [t.detach() for ws in weights for t in ws]
    dev = _require_hip(init_param, *flat)
    flat = [t if t.is_contiguous() and t.dtype == F32 else t.contiguous().to(F32) for t in flat]
    if len(flat) != 6 * (dim - 1):
        raise ValueError("fused_ar_pack: need 6 tensors per conditioner 1 .. dim-1")
    table = torch.tensor([t.data_ptr() for t in flat], dtype=torch.int64, device=dev)
    init = init_param.detach().to(F32).contiguous()
    n = int(_lib.load().nfk_fused_ar_pack_elems(dim, hidden, K))
    if n <= 0:
        raise ValueError("nfk_fused_ar: shape not supported")
    pack = torch.empty(n, dtype=F32, device=dev)
    _lib.call("nfk_fused_ar_pack", table.data_ptr(), init.data_ptr(), dim, hidden, K, pack.data_ptr(),
              _stream(dev))
    host = (ctypes.c_void_p * len(flat))(*[t.data_ptr() for t in flat])
    return pack, (table, init, flat, host)


def fused_ar(x, pack, dim, hidden, K, tail_bound, out, *, logdet, logdet_mode, inverse=False, status=None,
             split=True):
    """One fused NSF_AR layer (include/nfk.h nfk_fused_ar_ws).  split=False:
    no column split (the nfk_fused_ar launch) where the shape has the
    register form; the streamed-only shapes (fused_ar_inverse_supported
    False) always take their workspace, and a batch whose workspace exceeds
    config.AR_WORKSPACE_BYTES runs over row blocks."""
    dev = _require_hip(x, pack, out, logdet, status)
    B = x.shape[0]
    if x.dim() != 2 or x.shape[1] != dim or out.shape != x.shape:
        raise ValueError("fused_ar: x and out must be [B, %d]" % dim)
    lib = _lib.load()
    streamed = not bool(lib.nfk_fused_ar_inverse_supported(dim, hidden, K))
    if streamed and inverse:
        raise ValueError("fused_ar: the inverse of this shape is not fused (fused_ar_inverse_supported)")
    # a batch too small to fill the GPU splits the forward's conditioners over
    # workgroups; the per-column log|det| terms go through a workspace (and the
    # streamed form's trig operands)
    nws = int(lib.nfk_fused_ar_workspace(dim, hidden, K, B, 1 if inverse else 0)) if (split or streamed) else 0
    if streamed and 4 * nws > config.AR_WORKSPACE_BYTES and B > 64:
        rows = max(64, int(config.AR_WORKSPACE_BYTES // (4 * nws / B)) // 64 * 64)
        if rows < B:
            for r0 in range(0, B, rows):
                r1 = min(B, r0 + rows)
                fused_ar(x[r0:r1], pack, dim, hidden, K, tail_bound, out[r0:r1],
                         logdet=None if logdet is None else logdet[r0:r1], logdet_mode=logdet_mode,
                         status=status, split=split)
            return
    xp, ldx = _mat(x, "x")
    op, ldo = _mat(out, "out")
    ws = torch.empty(nws, dtype=F32, device=dev) if nws > 0 else None
    _timed("nfk_fused_ar", dev, "nfk_fused_ar_ws", xp, ldx, pack.data_ptr(), dim, hidden, K, float(tail_bound),
           op, ldo, _vec(logdet, B, "logdet"), logdet_mode, B, 1 if inverse else 0,
           _vec(status, dim, "status", torch.int32), None if ws is None else ws.data_ptr(), nws, _stream(dev))


def fused_nsf_supported(n_lo, n_up, hidden, K):
    return bool(_lib.load().nfk_fused_nsf_supported(n_lo, n_up, hidden, K))


def fused_nsf_pack(w0, b0, w2, b2, w4, b4, n_lo, n_up, hidden, K):
    dev = _require_hip(w0, b0, w2, b2, w4, b4)
    n = int(_lib.load().nfk_fused_nsf_pack_elems(n_lo, n_up, hidden, K))
    pack = torch.empty(n, dtype=F32, device=dev)
    ws = [t.detach().contiguous() for t in (w0, b0, w2, b2, w4, b4)]
    _lib.call("nfk_fused_nsf_pack", *[t.data_ptr() for t in ws], n_lo, n_up, hidden, K,
              pack.data_ptr(), _stream(dev))
    return pack


def fused_nsf(x, wpack, up_in, up_out, lo_in, lo_out, hidden, z, *, logdet, logdet_mode, K,
              tail_bound, inverse=False, status=None):
    dev = _require_hip(x, wpack, up_in, z, logdet, status)
    B = x.shape[0]
    xp, ldx = _mat(x, "x")
    zp, ldz = _mat(z, "z")
    # wide conditioners (k_fused_cl) on a small batch split their upper
    # coordinates over workgroups; the per-coordinate log|det| terms go through
    # a workspace (0 floats for every other shape)
    nws = int(_lib.load().nfk_fused_nsf_workspace(lo_in.numel(), up_in.numel(), hidden, K, B,
                                                  1 if inverse else 0))
    ws = torch.empty(nws, dtype=F32, device=dev) if nws > 0 else None
    _timed("nfk_fused_nsf", dev, "nfk_fused_nsf_ws", xp, ldx, wpack.data_ptr(), up_in.data_ptr(),
           up_out.data_ptr(), up_in.numel(), lo_in.data_ptr(), lo_out.data_ptr(), lo_in.numel(), hidden, zp, ldz,
           _vec(logdet, B, "logdet"), logdet_mode, B, K, float(tail_bound),
           1 if inverse else 0, _vec(status, 1, "status", torch.int32),
           None if ws is None else ws.data_ptr(), nws, _stream(dev))


_VJP_ELEMS = {}


def fused_nsf_vjp_supported(n_lo, n_up, hidden, K):
    key = (n_lo, n_up, hidden, K)
    n = _VJP_ELEMS.get(key)
    if n is None:
        n = _VJP_ELEMS[key] = int(_lib.load().nfk_fused_nsf_vjp_pack_elems(n_lo, n_up, hidden, K))
    return n > 0


def fused_nsf_vjp_pack(w0, b0, w2, b2, w4, b4, n_lo, n_up, hidden, K):
    dev = _require_hip(w0, b0, w2, b2, w4, b4)
    n = int(_lib.load().nfk_fused_nsf_vjp_pack_elems(n_lo, n_up, hidden, K))
    if n <= 0:
        raise ValueError("nfk_fused_nsf_vjp: shape not supported")
    ws = [t.detach().contiguous() for t in (w0, b0, w2, b2, w4, b4)]
    pack = torch.empty(n, dtype=F32, device=dev)
    _lib.call("nfk_fused_nsf_vjp_pack", *[t.data_ptr() for t in ws], n_lo, n_up, hidden, K, pack.data_ptr(),
              _stream(dev))
    return pack


def fused_nsf_vjp(x, vpack, up_in, up_out, lo_in, lo_out, hidden, gz, gld, gparams, gx, h1, h2, *, K,
                  tail_bound, inverse=False):
    """Recompute + spline VJP of one fused NSF_CL layer (include/nfk.h nfk_fused_nsf_vjp).
    h1, h2: [B, ldh] with ldh >= hidden + 1 (a multiple of 4); gparams [B, n_up*(3K-1)]."""
    dev = _require_hip(x, vpack, up_in, gz, gld, gparams, gx, h1, h2)
    B = x.shape[0]
    n_up, n_lo = up_in.numel(), lo_in.numel()
    xp, ldx = _mat(x, "x")
    gzp, ldgz = _mat(gz, "gz") if gz is not None else (None, 0)
    gxp, ldgx = _mat(gx, "gx")
    if gparams.shape != (B, n_up * (3 * K - 1)) or not gparams.is_contiguous():
        raise ValueError("gparams must be a contiguous [%d, %d] tensor" % (B, n_up * (3 * K - 1)))
    h1p, ldh = _mat(h1, "h1")
    h2p, ldh2 = _mat(h2, "h2")
    if ldh2 != ldh or h1.shape[1] < hidden + 1:
        raise ValueError("h1 and h2 need one row stride and hidden + 1 columns")
    _timed("nfk_fused_nsf_vjp", dev, "nfk_fused_nsf_vjp", xp, ldx, vpack.data_ptr(), up_in.data_ptr(),
           up_out.data_ptr(), n_up, lo_in.data_ptr(), lo_out.data_ptr(), n_lo, hidden, gzp, ldgz,
           _vec(gld, B, "gld"), gparams.data_ptr(), gxp, ldgx, h1p, h2p, ldh, B, K, float(tail_bound),
           1 if inverse else 0, _stream(dev))


_CHAIN_MAX = {}


def fused_nsf_chain_max(n_lo, n_up, hidden, K):
    """Most NSF_CL layers of this shape one nfk_fused_nsf_chain launch holds (0: none)."""
    key = (n_lo, n_up, hidden, K)
    n = _CHAIN_MAX.get(key)
    if n is None:
        n = _CHAIN_MAX[key] = int(_lib.load().nfk_fused_nsf_chain_max(n_lo, n_up, hidden, K))
    return n


def fused_nsf_chain(x, wpacks, cmaps, nlayers, n_lo, n_up, hidden, z, *, logdet, logdet_mode, K,
                    tail_bound, inverse=False, status=None, log_prob=None, prior_scale=1.0,
                    prior_hld=0.0):
    """nlayers fused NSF_CL layers in one launch (include/nfk.h nfk_fused_nsf_chain).
    wpacks: int64 device tensor of the layers' pack pointers; cmaps: int32 device
    tensor [nlayers * D + D] of composed tile columns; status: nlayers words.
    log_prob (optional [batch]): the isotropic-normal prior epilogue, z may be None."""
    dev = _require_hip(x, wpacks, cmaps, z, logdet, status, log_prob)
    B = x.shape[0]
    D = n_lo + n_up
    if wpacks.dtype != torch.int64 or wpacks.numel() != nlayers:
        raise ValueError("wpacks must hold %d int64 pack pointers" % nlayers)
    _vec(cmaps, nlayers * D + D, "cmaps", torch.int32)
    if x.dim() != 2 or x.shape[1] != D or (z is not None and tuple(z.shape) != tuple(x.shape)):
        raise ValueError("x and z must be [batch, %d] (n_lo + n_up) tensors" % D)
    xp, ldx = _mat(x, "x")
    zp, ldz = _mat(z, "z") if z is not None else (None, 0)
    _timed("nfk_fused_nsf_chain", dev, "nfk_fused_nsf_chain", xp, ldx, wpacks.data_ptr(), cmaps.data_ptr(),
           nlayers, n_lo, n_up, hidden, zp, ldz, _vec(logdet, B, "logdet"), logdet_mode, B, K,
           float(tail_bound), 1 if inverse else 0, _vec(status, nlayers, "status", torch.int32),
           _vec(log_prob, B, "log_prob"), float(prior_scale), float(prior_hld), _stream(dev))


_CHAIN_SAVED_OK = {}


def fused_nsf_chain_saved_ok(n_lo, n_up, hidden, K, nlayers):
    """Whether nfk_fused_nsf_chain_saved takes this shape and layer count."""
    key = (n_lo, n_up, hidden, K, nlayers)
    ok = _CHAIN_SAVED_OK.get(key)
    if ok is None:
        ok = _CHAIN_SAVED_OK[key] = bool(_lib.load().nfk_fused_nsf_chain_saved_ok(n_lo, n_up, hidden, K, nlayers))
    return ok


def fused_nsf_chain_saved(x, wpacks, cmaps, smaps, nlayers, n_lo, n_up, hidden, z, saves, *, logdet,
                          logdet_mode, K, tail_bound, status=None):
    """The training forward of a chain (include/nfk.h nfk_fused_nsf_chain_saved):
    z and log|det| of nlayers fused NSF_CL layers, and saves[l - 1] = the input
    of layer l >= 1 ([nlayers - 1, batch, D], contiguous rows); smaps: int32
    device tensor [(nlayers - 1) * D] of the tile columns of those inputs."""
    dev = _require_hip(x, wpacks, cmaps, smaps, z, saves, logdet, status)
    B = x.shape[0]
    D = n_lo + n_up
    if wpacks.dtype != torch.int64 or wpacks.numel() != nlayers:
        raise ValueError("wpacks must hold %d int64 pack pointers" % nlayers)
    _vec(cmaps, nlayers * D + D, "cmaps", torch.int32)
    _vec(smaps, (nlayers - 1) * D, "smaps", torch.int32)
    if saves.dtype != F32 or saves.dim() != 3 or tuple(saves.shape) != (nlayers - 1, B, D) or \
            saves.stride(2) != 1:
        raise ValueError("saves must be a float32 [%d, %d, %d] tensor with unit column stride"
                         % (nlayers - 1, B, D))
    if x.dim() != 2 or x.shape[1] != D or tuple(z.shape) != tuple(x.shape):
        raise ValueError("x and z must be [batch, %d] (n_lo + n_up) tensors" % D)
    xp, ldx = _mat(x, "x")
    zp, ldz = _mat(z, "z")
    _timed("nfk_fused_nsf_chain_saved", dev, "nfk_fused_nsf_chain_saved", xp, ldx, wpacks.data_ptr(),
           cmaps.data_ptr(), nlayers, n_lo, n_up, hidden, zp, ldz, _vec(logdet, B, "logdet"), logdet_mode, B, K,
           float(tail_bound), _vec(status, nlayers, "status", torch.int32), saves.data_ptr(), saves.stride(1),
           saves.stride(0), smaps.data_ptr(), _stream(dev))


def fused_realnvp_supported(half_dim, hidden):
    return bool(_lib.load().nfk_fused_realnvp_supported(half_dim, hidden))


def fused_realnvp_pack(nets, half_dim, hidden):
    """nets: 24 tensors, s1, t1, s2, t2 each (W0, b0, W2, b2, W4, b4)."""
    dev = _require_hip(*nets)
    n = int(_lib.load().nfk_fused_realnvp_pack_elems(half_dim, hidden))
    pack = torch.empty(n, dtype=F32, device=dev)
    ws = [t.detach().contiguous() for t in nets]
    ptrs = (ctypes.c_void_p * 24)(*[t.data_ptr() for t in ws])
    _lib.call("nfk_fused_realnvp_pack", ctypes.cast(ptrs, ctypes.c_void_p), half_dim, hidden, pack.data_ptr(),
              _stream(dev))
    return pack


_RCHAIN_MAX = {}


def fused_realnvp_chain_max(half_dim, hidden):
    """Most RealNVP layers of this shape one nfk_fused_realnvp_chain launch holds (0: none)."""
    key = (half_dim, hidden)
    n = _RCHAIN_MAX.get(key)
    if n is None:
        n = _RCHAIN_MAX[key] = int(_lib.load().nfk_fused_realnvp_chain_max(half_dim, hidden))
    return n


def fused_realnvp_chain(x, wpacks, nlayers, half_dim, hidden, z, *, logdet, logdet_mode, inverse=False,
                        status=None, log_prob=None, prior_scale=1.0, prior_hld=0.0):
    """nlayers fused RealNVP layers in one launch (include/nfk.h nfk_fused_realnvp_chain).
    wpacks: int64 device tensor of the layers' pack pointers in execution order;
    log_prob (optional [batch]): the isotropic-normal prior epilogue, z may be None."""
    dev = _require_hip(x, wpacks, z, logdet, status, log_prob)
    B = x.shape[0]
    if wpacks.dtype != torch.int64 or wpacks.numel() != nlayers:
        raise ValueError("wpacks must hold %d int64 pack pointers" % nlayers)
    xp, ldx = _mat(x, "x")
    zp, ldz = _mat(z, "z") if z is not None else (None, 0)
    _timed("nfk_fused_realnvp_chain", dev, "nfk_fused_realnvp_chain", xp, ldx, wpacks.data_ptr(), nlayers,
           half_dim, hidden, zp, ldz, _vec(logdet, B, "logdet"), logdet_mode, B, 1 if inverse else 0,
           _vec(status, 1, "status", torch.int32), _vec(log_prob, B, "log_prob"), float(prior_scale),
           float(prior_hld), _stream(dev))


def fused_realnvp(x, wpack, half_dim, hidden, z, *, logdet, logdet_mode, inverse=False):
    dev = _require_hip(x, wpack, z, logdet)
    B = x.shape[0]
    xp, ldx = _mat(x, "x")
    zp, ldz = _mat(z, "z")
    _timed("nfk_fused_realnvp", dev, "nfk_fused_realnvp", xp, ldx, wpack.data_ptr(), half_dim, hidden, zp, ldz,
           _vec(logdet, B, "logdet"), logdet_mode, B, 1 if inverse else 0, _stream(dev))


# ---- RealNVP with wide conditioners at small batches (nfk_wide_rnvp.hip)
def wlin_pack(W):
    """An nn.Linear weight [N, K] as the weight-streaming pack (nfk_wlin_pack:
    fp16 hi/lo MFMA fragments, one power-of-two scale, a zero block)."""
    dev = _require_hip(W)
    W = W.detach()
    if W.dtype != F32 or not W.is_contiguous():
        W = W.contiguous().to(F32)
    if W.dim() != 2:
        raise ValueError("wlin_pack: W must be 2-D")
    N, K = W.shape
    n = int(_lib.load().nfk_wlin_pack_floats(N, K))
    if n <= 0:
        raise ValueError("wlin_pack: bad shape %s" % (tuple(W.shape),))
    pack = torch.empty(n, dtype=F32, device=dev)
    _lib.call("nfk_wlin_pack", W.data_ptr(), N, K, pack.data_ptr(), _stream(dev))
    return pack


def wide_rnvp_supported(half, hidden):
    return bool(_lib.load().nfk_wide_rnvp_supported(half, hidden))


class WideRnvpPack:
    """The twelve packed Linears and biases of one RealNVP layer for
    wide_rnvp, with their host pointer tables (built once)."""

    def __init__(self, packs, biases, half, hidden):
        if len(packs) != 12 or len(biases) != 12:
            raise ValueError("wide_rnvp: 12 packs and 12 biases")
        for b in biases:
            if b.dtype != F32 or not b.is_contiguous():
                raise ValueError("wide_rnvp: biases must be contiguous float32")
        self.packs, self.biases, self.half, self.hidden = packs, biases, half, hidden
        self.device = _require_hip(*packs, *biases)
        self._pk = (ctypes.c_void_p * 12)(*[t.data_ptr() for t in packs])
        self._bs = (ctypes.c_void_p * 12)(*[t.data_ptr() for t in biases])
        self.pk, self.bs = ctypes.addressof(self._pk), ctypes.addressof(self._bs)
        self._ws = {}

    def workspace_floats(self, batch):
        n = self._ws.get(batch)
        if n is None:
            n = self._ws[batch] = int(_lib.load().nfk_wide_rnvp_workspace(self.half, self.hidden, batch))
        return n


def wide_rnvp(x, wp, z, *, logdet, logdet_mode, inverse=False):
    """One RealNVP layer through the weight stream (include/nfk.h
    nfk_wide_rnvp); ``wp`` a WideRnvpPack (packs / biases index 6 c + 2 l + g:
    half-coupling c: 0 = s1/t1, 1 = s2/t2; Linear l = network.0, .2, .4;
    conditioner g: 0 = s, 1 = t)."""
    dev = _require_hip(x, z, logdet)
    if dev != wp.device:
        raise RuntimeError("wide_rnvp: x on %s, the pack on %s" % (dev, wp.device))
    B = x.shape[0]
    xp, ldx = _mat(x, "x")
    zp, ldz = _mat(z, "z")
    if x.shape[1] != 2 * wp.half or z.shape != x.shape:
        raise ValueError("wide_rnvp: x and z must be [B, %d]" % (2 * wp.half))
    nws = wp.workspace_floats(B)
    ws = torch.empty(max(nws, 4), dtype=F32, device=dev)
    _timed("nfk_wide_rnvp", dev, "nfk_wide_rnvp", xp, ldx, wp.pk, wp.bs, wp.half, wp.hidden, zp, ldz,
           _vec(logdet, B, "logdet"), logdet_mode, B, 1 if inverse else 0, ws.data_ptr(), nws, _stream(dev))


class WideRnvpChain:
    """Host pointer tables of a run of WideRnvpPacks in execution order (12
    packs and 12 biases per layer) for wide_rnvp_chain; built once per run."""

    def __init__(self, wps):
        if not wps or any(w.half != wps[0].half or w.hidden != wps[0].hidden or w.device != wps[0].device
                          for w in wps):
            raise ValueError("wide_rnvp_chain: layers of one shape and device")
        self.wps, self.n = list(wps), len(wps)
        self.half, self.hidden, self.device = wps[0].half, wps[0].hidden, wps[0].device
        self._pk = (ctypes.c_void_p * (12 * self.n))(*[t.data_ptr() for w in wps for t in w.packs])
        self._bs = (ctypes.c_void_p * (12 * self.n))(*[t.data_ptr() for w in wps for t in w.biases])
        self.pk, self.bs = ctypes.addressof(self._pk), ctypes.addressof(self._bs)
        self._ws = {}

    def workspace_floats(self, batch):
        n = self._ws.get(batch)
        if n is None:
            n = self._ws[batch] = int(_lib.load().nfk_wide_rnvp_chain_workspace(self.half, self.hidden, batch))
        return n


def wide_rnvp_chain(x, chain, z, *, logdet, logdet_mode, inverse=False):
    """``chain.n`` RealNVP layers through the weight stream in one call
    (include/nfk.h nfk_wide_rnvp_chain), bitwise the per-layer wide_rnvp
    calls; ``chain`` a WideRnvpChain in execution order."""
    dev = _require_hip(x, z, logdet)
    if dev != chain.device:
        raise RuntimeError("wide_rnvp_chain: x on %s, the packs on %s" % (dev, chain.device))
    B = x.shape[0]
    xp, ldx = _mat(x, "x")
    zp, ldz = _mat(z, "z")
    if x.shape[1] != 2 * chain.half or z.shape != x.shape:
        raise ValueError("wide_rnvp_chain: x and z must be [B, %d]" % (2 * chain.half))
    nws = chain.workspace_floats(B)
    ws = torch.empty(max(nws, 4), dtype=F32, device=dev)
    _timed("nfk_wide_rnvp_chain", dev, "nfk_wide_rnvp_chain", xp, ldx, chain.pk, chain.bs, chain.n, chain.half,
           chain.hidden, zp, ldz, _vec(logdet, B, "logdet"), logdet_mode, B, 1 if inverse else 0, ws.data_ptr(), nws,
           _stream(dev))


# ---- NSF_AR inverse, column by column from the library (nfk_ar_seqinv.hip)
def ar_seqinv_supported(dim, hidden, K):
    return bool(_lib.load().nfk_ar_seqinv_supported(dim, hidden, K))


def ar_seqinv(z, ptrs, init_param, dim, hidden, K, tail_bound, out, *, logdet, logdet_mode, status=None):
    """NSF_AR.inverse of one layer (include/nfk.h nfk_ar_seqinv): ``ptrs`` is
    the HOST array of the conditioners' Linear tensor pointers that
    fused_ar_pack returns (keep[3], 6 per conditioner)."""
    dev = _require_hip(z, init_param, out, logdet, status)
    B = z.shape[0]
    zp, ldz = _mat(z, "z")
    op, ldo = _mat(out, "out")
    if z.shape[1] != dim or out.shape != z.shape:
        raise ValueError("ar_seqinv: z and out must be [B, %d]" % dim)
    if not isinstance(ptrs, ctypes.Array) or len(ptrs) != 6 * (dim - 1):
        raise ValueError("ar_seqinv: ptrs must be a ctypes array of 6 (dim - 1) pointers (fused_ar_pack's keep[3])")
    lib = _lib.load()
    nws = int(lib.nfk_ar_seqinv_workspace(dim, hidden, K, B))
    ws = torch.empty(max(nws, 4), dtype=F32, device=dev)
    _timed("nfk_ar_seqinv", dev, "nfk_ar_seqinv", zp, ldz, ctypes.cast(ptrs, ctypes.c_void_p).value,
           _vec(init_param, 3 * K - 1, "init_param"),
           dim, hidden, K, float(tail_bound), op, ldo, _vec(logdet, B, "logdet"), logdet_mode, B,
           _vec(status, dim, "status", torch.int32), ws.data_ptr(), nws, _stream(dev))
