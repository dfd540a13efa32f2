"""CPU: the shipped gfx950 objects keep DESIGN.md section 10.5's rule -- no
MFMA kernel that two waves could share a SIMD with contains packed-FP32 VALU
instructions (normalizingflow_amd/_isacheck.py; build() enforces it too).
Skipped when the objects are not built in this tree."""
import glob
import os

import pytest

from normalizingflow_amd import _isacheck

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJS = sorted(glob.glob(os.path.join(ROOT, "build", "*.o")))

_needs_objs = pytest.mark.skipif(not OBJS or not os.path.exists(_isacheck.LLVM_BIN),
                                reason="objects or LLVM tools not present")


@_needs_objs
def test_no_packed_fp32_in_two_wave_mfma_kernels():
    assert _isacheck.violations(OBJS) == []


@_needs_objs
def test_scan_sees_the_kernels():
    """The scan is not vacuous: it finds the MFMA kernels, and the packed-FP32
    code the rule still allows sits only in one-wave-per-SIMD instances."""
    ar = _isacheck.scan(os.path.join(ROOT, "build", "nfk_fused_ar.o"))
    mfma = {k: r for k, r in ar.items() if r["mfma"]}
    assert len(mfma) >= 10
    packed = {k: r for k, r in mfma.items() if r["pk_f32"]}
    assert packed and all(_isacheck.one_wave_per_simd(r) for r in packed.values())
    chain = _isacheck.scan(os.path.join(ROOT, "build", "nfk_fused_chain2.o"))
    assert any(r["mfma"] for r in chain.values())
    assert not any(r["pk_f32"] for r in chain.values())


def test_notes_records_keep_their_own_counts():
    """The metadata keys are sorted, so a kernel's .agpr_count precedes its
    .name; argument records carry .name keys of their own."""
    text = """amdhsa.kernels:
  - .agpr_count:     0
    .args:
      - .name:           a
        .offset:         0
    .name:           k_first
    .vgpr_count:     120
  - .agpr_count:     92
    .args:
      - .name:           b
        .offset:         0
    .name:           k_second
    .vgpr_count:     328
amdhsa.target:   amdgcn-amd-amdhsa--gfx950
"""
    regs = _isacheck.parse_notes(text)
    assert regs == {"k_first": (120, 0), "k_second": (328, 92)}
    assert not _isacheck.one_wave_per_simd({"vgpr": 200, "agpr": 92})  # 200 in total: two waves fit
    assert _isacheck.one_wave_per_simd({"vgpr": 328, "agpr": 92})
