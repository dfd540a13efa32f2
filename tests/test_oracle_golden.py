"""Pin the CPU oracle to the reference: oracle(inputs, weights) == golden outputs.

The golden outputs were produced by the reference code itself
(tests/golden/make_golden.py).  The oracle runs the same torch CPU fp32 ops in
the same order, so agreement is expected to the last few ulps.
"""
import pytest
import torch

import golden_io as gio
from oracle import nf_oracle as orc

RT, AT = 2e-6, 2e-6  # oracle vs reference: same torch CPU ops, ulp-level slack


def _close(a, b, rtol=RT, atol=AT):
    torch.testing.assert_close(a, b, rtol=rtol, atol=atol, equal_nan=True)


@pytest.mark.parametrize("name", gio.names("rqs_"))
def test_rqs_fixture(name):
    meta, d, _ = gio.load(name)
    tb = meta["tail_bound"]
    y, lad = orc.unconstrained_rq_spline(d["x"], d["uw"], d["uh"], d["ud"], tail_bound=tb)
    _close(y, d["y"]); _close(lad, d["lad"])
    yi, ladi = orc.unconstrained_rq_spline(d["y"], d["uw"], d["uh"], d["ud"], inverse=True,
                                           tail_bound=tb)
    _close(yi, d["inv_y"], atol=1e-5); _close(ladi, d["inv_lad"], atol=1e-5)
    y64, lad64 = orc.unconstrained_rq_spline(d["x"].double(), d["uw"].double(), d["uh"].double(),
                                             d["ud"].double(), tail_bound=tb)
    _close(y64, d["y_f64"], rtol=1e-12, atol=1e-12); _close(lad64, d["lad_f64"], rtol=1e-12, atol=1e-12)


LAYERS = [n for n in gio.names() if n.split("_")[0] in ("nsfcl", "realnvp", "planar", "radial", "nsfar", "nsfar1",
                                                               "maf", "actnorm", "onebyone")]


@pytest.mark.parametrize("name", LAYERS)
def test_layer_fixture(name):
    meta, d, sd = gio.load(name)
    spec = gio.layer_spec(meta)
    z, ld = orc.apply_layer(spec, d["x"], sd)
    # NSF_AR's log|det| sums dim fp32 terms whose logits come from library
    # GEMMs (their blocking, hence rounding, follows the thread count): its
    # slack grows with dim (the default 2e-6 up to 24 columns)
    ld_at = AT * max(1.0, meta["kwargs"].get("dim", 0) / 24.0) if meta["type"] == "NSF_AR" else AT
    _close(z, d["z"])
    if meta.get("sd_from_seed") and "ld_f64" in d:
        # the seeded applications-shape fixtures sum thousands of terms from
        # GEMMs whose blocking (rounding) follows the thread count: the oracle's
        # log|det| within the tolerance of the reference's, or its error against
        # the fixture's fp64 truth within 2x the reference's own (max and p99)
        try:
            _close(ld.expand_as(d["ld"]), d["ld"], atol=ld_at)
        except AssertionError:
            eo, er = (ld.double() - d["ld_f64"]).abs(), (d["ld"].double() - d["ld_f64"]).abs()
            assert eo.max() <= 2 * er.max() + AT and torch.quantile(eo, 0.99) <= 2 * torch.quantile(er, 0.99) + AT
    else:
        _close(ld.expand_as(d["ld"]), d["ld"], atol=ld_at)
    if "rt_x" in d:
        # NSF_AR's inverse is sequential (each inverted coordinate conditions the
        # next ones, flows.py:191-209): ulp-level spline differences propagate
        # through dim conditioners, so its slack grows with dim (1e-5 at 24)
        at = 1e-5 * max(1.0, meta["kwargs"].get("dim", 0) / 24.0) if meta["type"] == "NSF_AR" else 1e-5
        xi, ldi = orc.apply_layer(spec, d["z"], sd, inverse=True)
        _close(xi, d["rt_x"], atol=at); _close(ldi, d["rt_ld"], atol=at)
        xa, lda = orc.apply_layer(spec, d["x"], sd, inverse=True)
        _close(xa, d["inv_x"], atol=at); _close(lda, d["inv_ld"], atol=at)
    if "z_f64" in d:
        # the seeded applications-shape NSF_AR fixtures' fp64 companions ran with
        # fp64 as torch's default dtype (make_golden.py _f64_run: fp64 log_det
        # accumulator, and torch.tensor(np.pi) in fp64): the oracle likewise
        seeded = meta.get("sd_from_seed", False)
        prev = torch.get_default_dtype()
        if seeded:
            torch.set_default_dtype(torch.float64)
        try:
            sd64 = {k: v.double() for k, v in sd.items()}
            z64, ld64 = orc.apply_layer(spec, d["x"].double(), sd64)
            _close(z64, d["z_f64"], rtol=1e-12, atol=1e-12)
            if seeded:
                _close(ld64, d["ld_f64"], rtol=1e-10, atol=1e-10)
                for src, o, l in ((d["z"], "rt_x", "rt_ld"), (d["x"], "inv_x", "inv_ld")):
                    xi64, ldi64 = orc.apply_layer(spec, src.double(), sd64, inverse=True)
                    _close(xi64, d[o + "_f64"], rtol=1e-10, atol=1e-10)
                    _close(ldi64, d[l + "_f64"], rtol=1e-10, atol=1e-10)
            else:
                # the reference accumulates NSF_CL's log_det in an fp32 zeros() buffer (flows.py:228)
                _close(ld64.to(d["ld_f64"].dtype).expand_as(d["ld_f64"]), d["ld_f64"], rtol=1e-6, atol=1e-5)
        finally:
            torch.set_default_dtype(prev)


def _model_specs(meta):
    return [dict(gio.layer_spec(dict(type=l["type"], kwargs=l["kwargs"])), prefix="flows.%d." % i)
            for i, l in enumerate(meta["layers"])]


@pytest.mark.parametrize("name", gio.names("model_"))
def test_model_fixture(name):
    meta, d, sd = gio.load(name)
    specs = _model_specs(meta)
    z, plp, ld = orc.model_forward(specs, sd, d["x"], meta["var"])
    _close(z, d["z"]); _close(plp, d["prior_lp"]); _close(ld, d["ld"], atol=1e-5)
    _close(plp + ld, d["log_prob"], atol=1e-5)
    if "rt_x" in d:
        xi, ldi = orc.model_inverse(specs, sd, d["z"])
        _close(xi, d["rt_x"], atol=1e-5); _close(ldi, d["rt_ld"], atol=1e-5)
        xs, lps, zs = orc.model_sample_from(specs, sd, d["sample_z"], meta["var"])
        _close(xs, d["sample_x"], atol=1e-5); _close(lps, d["sample_log_px"], atol=1e-4)


def test_no_inside_raises():
    x = torch.full((4,), 10.0)
    w = torch.zeros(4, 8)
    with pytest.raises(RuntimeError):
        orc.unconstrained_rq_spline(x, w, w, torch.zeros(4, 7), tail_bound=3.0)


def test_bin_width_check():
    x = torch.zeros(4)
    w = torch.zeros(4, 2000)
    with pytest.raises(ValueError):
        orc.unconstrained_rq_spline(x, w, w, torch.zeros(4, 1999), tail_bound=3.0)


# ---- the reference's data-dependent errors (tests/golden/make_golden.py negdisc_cases)
def test_negative_discriminant_fixture():
    """utils.py:121: the reference asserts on this batch; the oracle must too,
    and on exactly the rows that assert one at a time."""
    meta, d, _ = gio.load("err_rqs_negdisc")
    tb = meta["tail_bound"]
    args = (d["x"], d["uw"], d["uh"], d["ud"])
    with pytest.raises(AssertionError):
        orc.unconstrained_rq_spline(*args, inverse=True, tail_bound=tb)
    bad = []
    for i in range(d["x"].shape[0]):
        try:
            orc.unconstrained_rq_spline(*(a[i:i + 1] for a in args), inverse=True, tail_bound=tb)
        except AssertionError:
            bad.append(i)
    assert bad == d["row_neg"].tolist()


def test_nan_conditioner_layer_fixture():
    """A NaN weight in psi's output layer: NaN at that coordinate in the
    forward (flows.py:227-239) and AssertionError in the inverse."""
    meta, d, sd = gio.load("err_nsfcl_nan")
    spec = gio.layer_spec(meta)
    z, ld = orc.apply_layer(spec, d["x"], sd)
    _close(z, d["z"]); _close(ld, d["ld"])
    with pytest.raises(AssertionError):
        orc.apply_layer(spec, d["x"], sd, inverse=True)


def test_nan_conditioner_model_fixture():
    """Model level: forward / evaluate raise ValueError (the prior's argument
    validation on a NaN z), inverse raises AssertionError."""
    meta, d, sd = gio.load("err_model_nan")
    specs = _model_specs(meta)
    assert (meta["forward_raises"], meta["inverse_raises"]) == ("ValueError", "AssertionError")
    with pytest.raises(ValueError):
        orc.model_forward(specs, sd, d["x"], meta["var"])
    with pytest.raises(AssertionError):
        orc.model_inverse(specs, sd, d["x"])
    z, ld = d["x"], torch.zeros(d["x"].shape[0])
    for s in specs:
        z, l = orc.apply_layer(s, z, sd)
        ld = ld + l
    _close(z, d["z"]); _close(ld, d["ld"], atol=1e-5)


def test_knife_edge_fixtures():
    """negdisc_*_edge: inputs 1-6 ulps under the steepest NSF_CL bins' top
    knots.  The reference asserted on none of them; the oracle (same torch
    CPU ops) must not either, and reproduces the reference's inverse."""
    meta, d, sd = gio.load("negdisc_nsfcl_edge")
    assert not bool(d["ref_asserts"])
    xi, ldi = orc.apply_layer(gio.layer_spec(meta), d["x"], sd, inverse=True)
    _close(xi, d["inv_x"]); _close(ldi, d["inv_ld"], atol=1e-4)
    meta, d, sd = gio.load("negdisc_model_edge")
    assert not bool(d["ref_asserts"])
    xm, ldm = orc.model_inverse(_model_specs(meta), sd, d["z"])
    _close(xm, d["inv_x"]); _close(ldm, d["inv_ld"], atol=1e-4)
