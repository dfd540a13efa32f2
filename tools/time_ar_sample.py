"""NSF_AR sampling at the applications' batches:
model.sample(n) (nf/models.py:31-35: prior draws, then the layers' inverse,
nf/flows.py:193-209) for Einstein/LJ (dim 96, H 354) and Fe (dim 162, H 354)
at test.py / fe.py's 500-row batches, and Polymer.yaml (dim 2048, H 100) at 40
rows; 2-layer models (the configs' nlayers).  Prints one JSON object with the
per-call time and the per-layer inverse time, and which path ran."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import nf.flows as nff  # noqa: E402
import nf.models as nfm  # noqa: E402
from normalizingflow_amd import kernels as K_  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    dev = torch.device("cuda:0")
    out = {}
    cases = [("einstein96", 96, 354, (32 / (8 * 1.28)) ** (1.0 / 3.0), 500, 5),
             ("fe162", 162, 354, 3 * 2.8841 / 2, 500, 5),
             ("polymer2048", 2048, 100, 0.5, 40, 1)]
    for name, dim, H, B, rows, reps in cases:
        torch.manual_seed(dim)
        flows = [nff.NSF_AR(dim=dim, K=32, B=B, hidden_dim=H) for _ in range(2)]
        model = nfm.NormalizingFlowModel(torch.distributions.MultivariateNormal(torch.zeros(dim), torch.eye(dim)),
                                         flows).to(dev)
        model.prior = torch.distributions.MultivariateNormal(torch.zeros(dim, device=dev), torch.eye(dim, device=dev))
        fused = K_.fused_ar_inverse_supported(dim, H, 32)
        t = timed(lambda: model.sample(rows), reps)
        z = torch.randn(rows, dim, device=dev) * 0.3
        with torch.no_grad():
            ti = timed(lambda: flows[0].inverse(z), reps)
            tf = timed(lambda: flows[0](z), reps)
        out[name] = {"rows": rows, "fused_inverse": bool(fused), "sample_ms": round(t, 3),
                     "inverse_per_layer_ms": round(ti, 3), "forward_per_layer_ms": round(tf, 3)}
        print(name, out[name], file=sys.stderr, flush=True)
        del model, flows
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
