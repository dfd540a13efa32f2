"""GPU: RealNVP at Polymer_rnvp.yaml's shape -- the configuration the
reference's only Polymer driver loads (applications/examples/polymer.py:29,
applications/input/Polymer_rnvp.yaml:8-9,16-18: 2048 coordinates, hidden 4000,
10 layers, batch 40; the driver's sample(100) and evaluate, polymer.py:37-41).

* forward / both inverses vs the reference's seeded fixture realnvp_d2048_h4000
  (also covered by test_gpu_parity.test_layer_vs_reference_golden);
* a 2-layer model's log_prob vs the oracle at the north star's rtol 1e-5, at
  the config's 40 rows and the driver's 100;
* sample(100): its log_px equals log_prob of the drawn x.
Tolerances as tests/test_gpu_parity.py (z rtol 1e-5 / atol 2e-5, log|det|
rtol 1e-5 / atol 5e-5 with the fp64 fallback of close_or_on_par)."""
import pytest
import torch

import golden_io as gio
import nf.flows as nff
import nf.models as nfm
from normalizingflow_amd import flush_status_checks
from oracle import nf_oracle as orc
from test_gpu_parity import LD_ATOL, LD_RTOL, Z_ATOL, Z_RTOL, close, close_or_on_par

pytestmark = pytest.mark.gpu

VAR = 0.1  # Polymer_rnvp.yaml:24 prior vars


def test_rnvp2048_layer_vs_reference_golden(hip_device):
    meta, d, sd = gio.load("realnvp_d2048_h4000")
    layer = gio.load_into(nff.RealNVP(**meta["kwargs"]), sd).to(hip_device)
    with torch.no_grad():
        z, ld = layer(d["x"].to(hip_device))
        close(z, d["z"], Z_RTOL, Z_ATOL)
        close_or_on_par(ld, d["ld"], d["ld_f64"], LD_RTOL, LD_ATOL)
        xi, ldi = layer.inverse(d["z"].to(hip_device))
        close(xi, d["rt_x"], Z_RTOL, 5e-5)
        close_or_on_par(ldi, d["rt_ld"], d["rt_ld_f64"], LD_RTOL, LD_ATOL)
        xa, lda = layer.inverse(d["x"].to(hip_device))
        close(xa, d["inv_x"], Z_RTOL, 5e-5)
        close_or_on_par(lda, d["inv_ld"], d["inv_ld_f64"], LD_RTOL, LD_ATOL)
    # inverse(forward(x)) = x (RealNVP's inverse is exact, flows.py:65-76)
    assert float((xi - d["x"].to(hip_device)).abs().max()) < 1e-5


@pytest.fixture(scope="module")
def model2(hip_device):
    torch.manual_seed(2048)
    flows = [nff.RealNVP(2048, hidden_dim=4000) for _ in range(2)]
    prior = torch.distributions.MultivariateNormal(torch.zeros(2048), VAR * torch.eye(2048))
    model = nfm.NormalizingFlowModel(prior, flows)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    model = model.to(hip_device)
    model.prior = torch.distributions.MultivariateNormal(torch.zeros(2048, device=hip_device),
                                                        VAR * torch.eye(2048, device=hip_device))
    return model, sd


@pytest.mark.parametrize("rows", [40, 100])
def test_rnvp2048_model_log_prob_vs_oracle(rows, model2, hip_device):
    model, sd = model2
    specs = orc.realnvp_specs(2, 2048)
    x = torch.randn(rows, 2048, generator=torch.Generator().manual_seed(rows)) * VAR ** 0.5
    with torch.no_grad():
        ref = orc.model_log_prob(specs, sd, x, prior_var=VAR)
        lp = model.log_prob(x.to(hip_device))
    close(lp, ref, 1e-5, 1e-5)
    flush_status_checks()


def test_rnvp2048_sample(model2, hip_device):
    model, sd = model2
    xs, lpx, zs = model.sample(100)
    with torch.no_grad():
        lp = model.log_prob(xs)
    close(lpx, lp, 1e-5, 1e-3)
    ref_x, ref_lpx, _ = orc.model_sample_from(orc.realnvp_specs(2, 2048), sd, zs.cpu(), prior_var=VAR)
    close(xs, ref_x, Z_RTOL, 5e-5)
    close(lpx, ref_lpx, 1e-5, 1e-3)
    flush_status_checks()
