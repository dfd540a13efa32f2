"""Polymer_rnvp.yaml's flow on the GPU (applications/input/Polymer_rnvp.yaml:
RealNVP(2048, hidden 4000) x 10 at the config's 40-row batch; the driver's
sample(100) / evaluate at 100 rows, applications/examples/polymer.py:37-41):
log_prob and sample times, the per-GEMM time of one conditioner layer, and the
HBM floor of streaming the weights (4 x 24.2 M parameters per layer)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import nf.flows as nff  # noqa: E402
import nf.models as nfm  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    dev = torch.device("cuda:0")
    D, H, L = 2048, 4000, 10
    torch.manual_seed(1234)
    flows = [nff.RealNVP(D, hidden_dim=H) for _ in range(L)]
    prior = torch.distributions.MultivariateNormal(torch.zeros(D), 0.1 * torch.eye(D))
    model = nfm.NormalizingFlowModel(prior, flows).to(dev)
    model.prior = torch.distributions.MultivariateNormal(torch.zeros(D, device=dev), 0.1 * torch.eye(D, device=dev))
    wbytes = 4 * sum(p.numel() for p in model.parameters())
    floor_ms = wbytes / 8e12 * 1e3
    out = {"weights_bytes": wbytes, "hbm_floor_ms_per_step": floor_ms}
    from normalizingflow_amd import config
    from normalizingflow_amd import kernels as K_
    with torch.no_grad():
        for wide in (True, False):
            config.USE_WIDE_RNVP = wide
            tag = "wide" if wide else "library"
            for rows in (40, 100, 500):
                x = torch.randn(rows, D, device=dev) * 0.1 ** 0.5
                t = timed(lambda: model.log_prob(x))
                out["%s_log_prob_%d_ms" % (tag, rows)] = t
                out["%s_log_prob_%d_frac_of_hbm_floor" % (tag, rows)] = floor_ms / t
            out["%s_sample_100_ms" % tag] = timed(lambda: model.sample(100), 10)
        config.USE_WIDE_RNVP = True
        # per-layer call time of the weight stream (HIP events around each call)
        x = torch.randn(40, D, device=dev) * 0.1 ** 0.5
        K_.TIMER = K_.KernelTimer()
        for _ in range(5):
            model.log_prob(x)
        torch.cuda.synchronize()
        out["wide_layer_call_40"] = {k: {"calls": v[0], "mean_ms": v[1]} for k, v in K_.TIMER.summary().items()}
        K_.TIMER = None
        # one conditioner's three GEMMs at 40 rows (torch Linear: library GEMM)
        net = flows[0].s1
        x = torch.randn(40, D // 2, device=dev)
        w1, w2, w3 = net.network[0], net.network[2], net.network[4]
        h1 = torch.tanh(w1(x))
        h2 = torch.tanh(w2(h1))
        for name, fn, nb in (("gemm1_1024x4000", lambda: w1(x), 4 * (1024 * 4000 + 4000)),
                             ("gemm2_4000x4000", lambda: w2(h1), 4 * (4000 * 4000 + 4000)),
                             ("gemm3_4000x1024", lambda: w3(h2), 4 * (4000 * 1024 + 1024)),
                             ("fcnn", lambda: net(x), 4 * sum(p.numel() for p in net.parameters()))):
            t = timed(fn, 50)
            out[name + "_ms"] = t
            out[name + "_gbs"] = nb / (t * 1e-3) / 1e9
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
