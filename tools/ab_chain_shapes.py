"""A/B: log_prob of 8-layer NSF_CL models of several shapes through the chained
launch vs one fused launch per layer (config.USE_CHAIN), wall time per call."""
import sys, time, torch
sys.path.insert(0, '.')
import nf.flows as nff, nf.models as nfm
from normalizingflow_amd import config
dev = torch.device('cuda', 0)
for (size, K, H) in [(32, 8, 100), (32, 8, 128), (32, 8, 64), (32, 6, 130), (32, 10, 100)]:
    torch.manual_seed(0)
    flows = [nff.NSF_CL(size=size, dim=2, K=K, B=3, hidden_dim=H, mask=[i % 2]) for i in range(8)]
    D = 2 * size
    m = nfm.NormalizingFlowModel(torch.distributions.MultivariateNormal(torch.zeros(D), torch.eye(D)), flows).to(dev)
    m.prior = torch.distributions.MultivariateNormal(torch.zeros(D, device=dev), torch.eye(D, device=dev))
    x = torch.randn(1 << 20, D, device=dev)
    res = []
    for chain in (True, False, True, False):
        config.USE_CHAIN = chain
        for _ in range(2): m.log_prob(x)
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(5): m.log_prob(x)
        torch.cuda.synchronize(); res.append((time.perf_counter() - t0) / 5 * 1e3)
    print("size %d K %d H %d: chain %.2f/%.2f ms, per-layer %.2f/%.2f ms" % (size, K, H, res[0], res[2], res[1], res[3]), flush=True)
