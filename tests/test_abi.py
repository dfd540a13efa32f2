"""CPU checks of the C-ABI boundary: libnfk.so loads (no GPU needed to dlopen),
exports every symbol include/nfk.h declares, and the ctypes table matches."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "nfk.h")


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z0-9_]+\s*\*?\s*(nfk_[a-z0-9_]+)\s*\(",
                                 src, flags=re.M)))


def test_header_parses():
    syms = header_symbols()
    assert "nfk_rqs_coupling" in syms and "nfk_fused_nsf" in syms
    assert len(syms) >= 14


def test_library_exports_every_header_symbol():
    from normalizingflow_amd import _lib
    assert os.path.exists(_lib.LIB_PATH), "build libnfk.so first (__graft_entry__.build())"
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_ctypes_table_matches_header():
    from normalizingflow_amd import _lib
    assert sorted(_lib.SIGNATURES) == header_symbols()


def test_abi_version_and_host_only_calls():
    from normalizingflow_amd import _lib
    lib = _lib.load()
    assert lib.nfk_abi_version() == _lib.ABI_VERSION
    assert lib.nfk_radial_workspace_elems() > 0
    # argument validation runs on the host and never touches the device
    rc = lib.nfk_rqs_coupling(None, 0, None, None, None, 0, None, None, 0, None, 0, None, 0,
                              None, 0, 0, 8, -3.0, 3.0, -3.0, 3.0, 1, 1e-3, 1e-3, 1e-3, 0, 0,
                              None, None)
    assert rc == _lib.NFK_EINVAL
    assert b"bad sizes" in lib.nfk_last_error()
    rc = lib.nfk_rqs_coupling(1, 1, 1, 1, 1, 1, None, None, 0, 1, 1, None, 0, None, 0, 4, 2000,
                              -3.0, 3.0, -3.0, 3.0, 1, 1e-3, 1e-3, 1e-3, 0, 0, None, None)
    assert rc == _lib.NFK_EINVAL and b"bin width" in lib.nfk_last_error()


def test_fused_shape_query_is_host_only():
    from normalizingflow_amd import _lib
    lib = _lib.load()
    n = lib.nfk_fused_nsf_pack_elems(32, 32, 100, 8)
    sup = lib.nfk_fused_nsf_supported(32, 32, 100, 8)
    assert (sup == 0 and n == 0) or (sup == 1 and n > 0)
