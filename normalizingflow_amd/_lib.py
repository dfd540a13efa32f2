"""ctypes binding of libnfk.so (include/nfk.h).

The product path has no CPU or eager-PyTorch fallback: if the HIP library is
missing or was built for a different ABI, every call raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NFK_LIBRARY", os.path.join(_HERE, "libnfk.so"))
ABI_VERSION = 2

NFK_EINVAL = -1
ST_INSIDE_SEEN = 1
ST_NEG_DISC = 2
ST_NAN_Z = 4

P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
F64 = ctypes.c_double
F32 = ctypes.c_float

# name -> (restype, argtypes); mirrors include/nfk.h one-to-one
SIGNATURES = {
    "nfk_abi_version": (ctypes.c_int, []),
    "nfk_last_error": (ctypes.c_char_p, []),
    "nfk_maf": (ctypes.c_int, [
        P, I64, P, P, I64,              # x, ldx, init_param, params, ldp
        I32, I32, I32, P, I64,          # c0, c1, dim, out, ldo
        P, I32, I64, I32, P]),          # logdet, logdet_mode, batch, inverse, stream
    "nfk_actnorm": (ctypes.c_int, [
        P, I64, P, P, I32, P, I64,      # x, ldx, mu, log_sigma, dim, z, ldz
        P, I32, P, I64, I32, P]),       # logdet, logdet_mode, ld_scalar, batch, inverse, stream
    "nfk_rqs_coupling_bwd": (ctypes.c_int, [
        P, I64, P,                      # x, ldx, params
        P, P, I32,                      # up_in, up_out, n_up
        P, P, I32,                      # lo_in, lo_out, n_lo
        P, I64, P,                      # gz, ldgz, glogdet
        P, P, I64, I64, I32,            # gparams, gx, ldgx, batch, K
        F64, F64, F64, F64, I32,        # left, right, bottom, top, tails
        F64, F64, F64,                  # min_bin_width, min_bin_height, min_derivative
        I32, I32, P]),                  # param_mode, inverse, stream
    "nfk_rqs_coupling": (ctypes.c_int, [
        P, I64, P,                      # x, ldx, params
        P, P, I32,                      # up_in, up_out, n_up
        P, P, I32,                      # lo_in, lo_out, n_lo
        P, I64, P, I32,                 # z, ldz, logdet, logdet_mode
        P, I64, I64, I32,               # lad_out, ld_lad, batch, K
        F64, F64, F64, F64, I32,        # left, right, bottom, top, tails
        F64, F64, F64,                  # min_bin_width, min_bin_height, min_derivative
        I32, I32, P, P]),               # param_mode, inverse, status, stream
    "nfk_searchsorted": (ctypes.c_int, [P, P, P, I64, I32, F64, P]),
    "nfk_affine_coupling": (ctypes.c_int, [P, I64, P, P, I64, P, I64, P, I32, I64, I32, I32, P]),
    "nfk_planar": (ctypes.c_int, [P, I64, P, P, P, P, I64, P, I32, P, I64, I32, I32, P]),
    "nfk_radial_workspace_elems": (ctypes.c_int64, []),
    "nfk_radial_sumsq": (ctypes.c_int, [P, I64, P, I64, I32, P, P, P]),
    "nfk_radial_apply": (ctypes.c_int, [P, I64, P, P, P, P, P, I64, P, P, I32, I64, I32, P]),
    "nfk_normal_logprob": (ctypes.c_int, [P, I64, P, P, I64, I32, F32, F32, I32, P, P]),
    "nfk_trig_features": (ctypes.c_int, [P, I64, P, I64, I64, I32, F64, P]),
    "nfk_fused_ar_supported": (ctypes.c_int, [I32, I32, I32]),
    "nfk_fused_ar_inverse_supported": (ctypes.c_int, [I32, I32, I32]),
    "nfk_fused_ar_pack_elems": (ctypes.c_int64, [I32, I32, I32]),
    "nfk_fused_ar_pack": (ctypes.c_int, [P, P, I32, I32, I32, P, P]),
    "nfk_fused_ar": (ctypes.c_int, [
        P, I64, P, I32, I32, I32,       # x, ldx, pack, dim, hidden, K
        F64, P, I64, P, I32,            # tail_bound, out, ldo, logdet, logdet_mode
        I64, I32, P, P]),               # batch, inverse, status, stream
    "nfk_gather_cols_ones": (ctypes.c_int, [P, I64, P, I32, I64, P, I64, P]),
    "nfk_fused_ar_workspace": (ctypes.c_int64, [I32, I32, I32, I64, I32]),
    "nfk_fused_ar_ws": (ctypes.c_int, [
        P, I64, P, I32, I32, I32,       # x, ldx, pack, dim, hidden, K
        F64, P, I64, P, I32,            # tail_bound, out, ldo, logdet, logdet_mode
        I64, I32, P, P, I64, P]),       # batch, inverse, status, workspace, workspace_floats, stream
    "nfk_fused_nsf_supported": (ctypes.c_int, [I32, I32, I32, I32]),
    "nfk_fused_nsf_pack_elems": (ctypes.c_int64, [I32, I32, I32, I32]),
    "nfk_fused_nsf_pack": (ctypes.c_int, [P, P, P, P, P, P, I32, I32, I32, I32, P, P]),
    "nfk_fused_nsf": (ctypes.c_int, [
        P, I64, P,                      # x, ldx, wpack
        P, P, I32,                      # up_in, up_out, n_up
        P, P, I32, I32,                 # lo_in, lo_out, n_lo, hidden
        P, I64, P, I32,                 # z, ldz, logdet, logdet_mode
        I64, I32, F64, I32, P, P]),     # batch, K, tail_bound, inverse, status, stream
    "nfk_fused_nsf_workspace": (ctypes.c_int64, [I32, I32, I32, I32, I64, I32]),
    "nfk_fused_nsf_ws": (ctypes.c_int, [
        P, I64, P, P, P, I32, P, P, I32, I32,   # x, ldx, wpack, up_in, up_out, n_up, lo_in, lo_out, n_lo, hidden
        P, I64, P, I32, I64, I32, F64, I32, P,  # z, ldz, logdet, mode, batch, K, tail_bound, inverse, status
        P, I64, P]),                            # workspace, workspace_floats, stream
    "nfk_fused_nsf_chain_max": (ctypes.c_int, [I32, I32, I32, I32]),
    "nfk_fused_nsf_chain": (ctypes.c_int, [
        P, I64, P, P, I32,              # x, ldx, wpacks, cmaps, nlayers
        I32, I32, I32,                  # n_lo, n_up, hidden
        P, I64, P, I32,                 # z, ldz, logdet, logdet_mode
        I64, I32, F64, I32, P,          # batch, K, tail_bound, inverse, status
        P, F32, F32, P]),               # log_prob, prior_scale, prior_half_log_det, stream
    "nfk_fused_nsf_chain_saved_ok": (ctypes.c_int, [I32, I32, I32, I32, I32]),
    "nfk_fused_nsf_chain_saved": (ctypes.c_int, [
        P, I64, P, P, I32,              # x, ldx, wpacks, cmaps, nlayers
        I32, I32, I32,                  # n_lo, n_up, hidden
        P, I64, P, I32,                 # z, ldz, logdet, logdet_mode
        I64, I32, F64, P,               # batch, K, tail_bound, status
        P, I64, I64, P, P]),            # saves, ld_saves, save_stride, smaps, stream
    "nfk_fused_nsf_vjp_pack_elems": (ctypes.c_int64, [I32, I32, I32, I32]),
    "nfk_fused_nsf_vjp_pack": (ctypes.c_int, [P, P, P, P, P, P, I32, I32, I32, I32, P, P]),
    "nfk_fused_nsf_vjp": (ctypes.c_int, [
        P, I64, P, P, P, I32,           # x, ldx, vpack, up_in, up_out, n_up
        P, P, I32, I32,                 # lo_in, lo_out, n_lo, hidden
        P, I64, P,                      # gz, ldgz, glogdet
        P, P, I64,                      # gparams, gx, ldgx
        P, P, I64,                      # h1, h2, ldh
        I64, I32, F64, I32, P]),        # batch, K, tail_bound, inverse, stream
    "nfk_fused_realnvp_supported": (ctypes.c_int, [I32, I32]),
    "nfk_fused_realnvp_pack_elems": (ctypes.c_int64, [I32, I32]),
    "nfk_fused_realnvp_pack": (ctypes.c_int, [P, I32, I32, P, P]),
    "nfk_fused_realnvp": (ctypes.c_int, [
        P, I64, P, I32, I32,            # x, ldx, wpack, half_dim, hidden
        P, I64, P, I32,                 # z, ldz, logdet, logdet_mode
        I64, I32, P]),                  # batch, inverse, stream
    "nfk_fcnn_dh_pack_floats": (ctypes.c_int64, [I32, I32]),
    "nfk_fcnn_dh_pack": (ctypes.c_int, [P, I32, I32, P, P]),
    "nfk_fcnn_dh": (ctypes.c_int, [P, I64, I32, P, P, I64, I32, P, I64, I64, I32, I64, P]),
    "nfk_fcnn_linear": (ctypes.c_int, [P, I64, I32, P, P, I32, I32, P, I64, I64, P]),
    "nfk_wlin_pack_floats": (ctypes.c_int64, [I32, I32]),
    "nfk_wlin_pack": (ctypes.c_int, [P, I32, I32, P, P]),
    "nfk_wide_rnvp_supported": (ctypes.c_int, [I32, I32]),
    "nfk_wide_rnvp_workspace": (ctypes.c_int64, [I32, I32, I64]),
    "nfk_wide_rnvp": (ctypes.c_int, [P, I64, P, P, I32, I32, P, I64, P, I32, I64, I32, P, I64, P]),
    "nfk_wide_rnvp_chain_workspace": (ctypes.c_int64, [I32, I32, I64]),
    "nfk_wide_rnvp_chain": (ctypes.c_int, [P, I64, P, P, I32, I32, I32, P, I64, P, I32, I64, I32, P, I64, P]),
    "nfk_ar_seqinv_supported": (ctypes.c_int, [I32, I32, I32]),
    "nfk_ar_seqinv_workspace": (ctypes.c_int64, [I32, I32, I32, I64]),
    "nfk_ar_seqinv": (ctypes.c_int, [P, I64, P, P, I32, I32, I32, ctypes.c_double, P, I64, P, I32, I64, P, P, I64,
                                     P]),
    "nfk_flows_bwd_workspace_bytes": (ctypes.c_int64, [I64, I32]),
    "nfk_planar_bwd": (ctypes.c_int, [
        P, I64, P, P, P,                # x, ldx, w, u, b
        P, I64, P, P, I64,              # gz, ldgz, glogdet, gx, ldgx
        P, P, P, P, I64, I32, I32, P]),  # gw, gu, gb, workspace, batch, dim, nonlinearity, stream
    "nfk_actnorm_bwd": (ctypes.c_int, [
        P, I64, P, P, I32,              # x, ldx, mu, log_sigma, dim
        P, I64, P, P, I64,              # gz, ldgz, gld_scalar, gx, ldgx
        P, P, P, I64, I32, P]),         # gmu, gls, workspace, batch, inverse, stream
    "nfk_radial_bwd_scalars": (ctypes.c_int, [
        P, I64, P, P, P, P,             # x, ldx, x0, log_alpha, beta, sumsq
        P, I64, P, P, P, I64, I32, P]),  # gz, ldgz, gld_scalar, scal, workspace, batch, dim, stream
    "nfk_radial_bwd_apply": (ctypes.c_int, [
        P, I64, P, P, I64, P,           # x, ldx, x0, gz, ldgz, scal
        P, I64, P, P, I64, I32, P]),    # gx, ldgx, gx0, workspace, batch, dim, stream
    "nfk_maf_bwd": (ctypes.c_int, [
        P, I64, P, P, I64,              # x, ldx, init_param, params, ldp
        P, I64, P, I32, I32, I32,       # gout, ldgo, glogdet, c0, c1, dim
        P, I64, P, I64, P, P,           # gx, ldgx, gparams, ldgp, ginit, workspace
        I64, I32, P]),                  # batch, inverse, stream
    "nfk_trig_features_bwd": (ctypes.c_int, [P, I64, P, I64, P, I64, I64, I32, F64, P]),
    "nfk_affine_coupling_bwd": (ctypes.c_int, [
        P, I64, P, P, I64,              # x_in, ld_in, s, t, ld_st
        P, I64, P,                      # g_out, ld_g, g_logdet
        P, I64, I32, P, P, I64,         # g_in, ld_gin, accumulate, g_s, g_t, ld_gst
        I64, I32, I32, P]),             # batch, n, inverse, stream
    "nfk_fused_realnvp_chain_max": (ctypes.c_int, [I32, I32]),
    "nfk_fused_realnvp_chain": (ctypes.c_int, [
        P, I64, P, I32,                 # x, ldx, wpacks, nlayers
        I32, I32,                       # half_dim, hidden
        P, I64, P, I32,                 # z, ldz, logdet, logdet_mode
        I64, I32, P,                    # batch, inverse, status
        P, F32, F32, P]),               # log_prob, prior_scale, prior_half_log_det, stream
}

_lock = threading.Lock()
_lib = None


class NfkError(RuntimeError):
    """A libnfk.so entry point returned an error code."""


def load():
    """Load (once) and return the library; raise if it is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                "normalizingflow_amd: HIP kernel library not found at %s -- build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (or `make -C "
                "normalizingflow_amd/csrc`); there is no CPU fallback." % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        ver = lib.nfk_abi_version()
        if ver != ABI_VERSION:
            raise ImportError("libnfk.so ABI %d != expected %d; rebuild" % (ver, ABI_VERSION))
        _lib = lib
    return _lib


def call(name, *args):
    """Invoke an entry point and turn a non-zero return into an exception."""
    rc = getattr(load(), name)(*args)
    if rc != 0:
        msg = load().nfk_last_error()
        msg = msg.decode() if msg else ""
        if rc == NFK_EINVAL:
            raise ValueError("%s: %s" % (name, msg))
        raise NfkError("%s failed (hipError %d): %s" % (name, rc, msg))
    return rc
