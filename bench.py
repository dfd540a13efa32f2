#!/usr/bin/env python
"""Throughput of the log_prob hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

A step = one NormalizingFlowModel.log_prob pass over one per-GPU batch of
synthetic x ~ N(0, I) already resident in HBM (c3: 8 NSF_CL RQS coupling
layers, D=64, K=8, H=100, B = 2^20 per GPU).  With N > 1 every rank owns its
own 2^20 rows (weak scaling, sample sharding, BASELINE config 4) and the step
ends with the NLL all-reduce of [sum log p, count] over RCCL.

Rank 0 prints ONE JSON line; `roofline` is computed for the dominant kernel
from HIP events recorded live around its launches inside the timed region, and
`cpu_baseline` times the CPU oracle (torch-CPU fp32 restatement of the
reference path) on a bounded sample of the same workload on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_HBM_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
PEAK_FP32_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (= vector) peak, dense
PEAK_FP16_TFLOPS = 16 * PEAK_FP32_TFLOPS  # MI355X_MICROARCH.md: F16/BF16 MFMA = 16x f32, ~2.5 PF dense

WORKLOADS = {
    # name: (description, layer type, kwargs, D, flops/sample/layer, HBM bytes/sample/layer)
    "c3": ("64-dim synthetic Gaussian, 8-layer NSF_CL RQS spline coupling (K=8 bins, H=100, "
           "mask [i%2], B=3), log_prob", "NSF_CL",
           dict(size=32, dim=2, K=8, B=3, hidden_dim=100), 64, 8),
    "c2": ("64-dim synthetic Gaussian, 8-layer RealNVP affine coupling (H=100), log_prob",
           "RealNVP", dict(dim=64, hidden_dim=100), 64, 8),
    "c5": ("256-dim synthetic Gaussian, 16-layer NSF_CL RQS spline coupling (K=16 bins, H=256, "
           "mask [i%2], B=3), log_prob", "NSF_CL",
           dict(size=128, dim=2, K=16, B=3, hidden_dim=256), 256, 16),
}


METRICS = {
    "c3": "samples/sec log_prob (1M×64, 8 RQS coupling layers) at 1/2/4/8 GPU",  # BASELINE.json
    "c2": "samples/sec log_prob (1M×64, 8 RealNVP affine coupling layers)",
    "c5": "samples/sec log_prob (1M×256, 16 RQS coupling layers, H=256, K=16)",
}


# conditioner arithmetic of the fused layer kernels per workload
_SPLIT = "fp16 two-way split (hi+lo, 3 MFMA products, fp32 accumulate, power-of-two pre-scaling)"
ARITH = {
    "c3": _SPLIT + "; 4-feature k-tail on f32 MFMA (nfk_fused_impl.h)",
    "c2": _SPLIT + "; 4-feature k-tail on f32 MFMA (nfk_fused_rnvp.hip)",
    "c5": _SPLIT + " (nfk_fused_wide.h)",
}


def build_model(workload, device):
    import nf.flows as nff
    import nf.models as nfm
    desc, kind, kw, D, L = WORKLOADS[workload]
    torch.manual_seed(1234)  # weights seed 1234, nn.Linear default init, on CPU
    if kind == "NSF_CL":
        flows = [nff.NSF_CL(mask=[i % 2], **kw) for i in range(L)]
    else:
        flows = [nff.RealNVP(**kw) for _ in range(L)]
    prior = torch.distributions.MultivariateNormal(torch.zeros(D), torch.eye(D))
    model = nfm.NormalizingFlowModel(prior, flows)
    cpu_model = model
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    model = model.to(device)
    model.prior = torch.distributions.MultivariateNormal(torch.zeros(D, device=device),
                                                        torch.eye(D, device=device))
    return model, sd, cpu_model


def specs_for(workload):
    from oracle import nf_oracle as orc
    desc, kind, kw, D, L = WORKLOADS[workload]
    if kind == "NSF_CL":
        return orc.nsf_cl_specs(L, kw["size"], kw["dim"], kw["K"], kw["B"], [[0], [1]])
    return orc.realnvp_specs(L, kw["dim"])


def cpu_baseline(workload, sd, budget_s=10.0):
    """Time the CPU oracle on a bounded sample (about budget_s of CPU work)."""
    from oracle import nf_oracle as orc
    D = WORKLOADS[workload][3]
    specs = specs_for(workload)
    g = torch.Generator().manual_seed(0)
    with torch.inference_mode():
        x = torch.randn(4096, D, generator=g)
        t0 = time.perf_counter()
        orc.model_log_prob(specs, sd, x)  # warm-up + rate estimate
        t_w = time.perf_counter() - t0
        n = int(max(4096, min(1 << 20, 4096 * budget_s / max(t_w, 1e-3))))
        n = (n // 4096) * 4096
        x = torch.randn(n, D, generator=g)
        t0 = time.perf_counter()
        orc.model_log_prob(specs, sd, x)
        dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "samples/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": "%s log_prob of %d x %d rows (seed 0) by the CPU oracle (oracle/nf_oracle.py: "
                      "torch-CPU fp32 restatement of nf/models.py:37 evaluate), %d threads, "
                      "1 warm-up + 1 timed run, %.1f s" % (workload, n, D,
                                                            torch.get_num_threads(), dt)}


def roofline(workload, timer_summary, per_gpu_batch, traffic, n_steps):
    """Roofline of the dominant kernel from live HIP-event timings."""
    if not timer_summary:
        return None
    name, (n_launch, mean_ms, tot) = max(timer_summary.items(), key=lambda kv: kv[1][2])
    n = n_launch
    desc, kind, kw, D, L = WORKLOADS[workload]
    B = per_gpu_batch
    if name in ("nfk_fused_nsf", "nfk_fused_nsf_chain"):
        # layers per launch: all L of a step in one chain launch (or one per launch)
        per = L * n_steps / n_launch if name == "nfk_fused_nsf_chain" else 1
        H = kw["hidden_dim"]
        n_lo = kw["size"]  # mask of one coordinate per particle (dim=2)
        n_up = kw["size"] * (kw["dim"] - 1)
        P = 3 * kw["K"] - 1
        # the kernel's formulation (nfk_fused_impl.h): every product runs as a
        # two-way fp16 split (3 MFMA products) except, when H = 32 KBH + R with
        # 0 < R <= 4, the R-feature k-tail of layers 2-3 on exact f32 MFMA
        kbf, R = divmod(H, 32)
        tail = R if (0 < R <= 4 and kbf >= 1) else 0
        f32 = 2.0 * tail * (H + n_up * P)
        f16 = 2.0 * (n_lo * H + H * H + H * n_up * P) - f32
        flops = (f16 + f32) * B * per            # 173,600/sample/layer (fp32-equivalent)
        # MFMA-time floor of this formulation at the dense peak of the MFMA each
        # part runs on, expressed as an fp32-equivalent TFLOP/s peak
        t_floor = f32 / (PEAK_FP32_TFLOPS * 1e12) + 3.0 * f16 / (PEAK_FP16_TFLOPS * 1e12)
        peak = (f16 + f32) / t_floor / 1e12
        achieved = flops / (mean_ms * 1e-3) / 1e12
        return {"kernel": name, "bound": "mfma", "achieved": round(achieved, 2),
                "peak": round(peak, 1), "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "launches": n, "mean_ms": round(mean_ms, 4),
                "per_launch": "%d samples x %g layers x %.0f flop (fp32-equivalent)"
                              % (B, per, flops / B / per),
                "peak_basis": "MFMA floor: %.0f flop/sample as 3 fp16 products (%.1f TF dense) + "
                              "%.0f flop/sample k-tail on f32 MFMA (%.1f TF)"
                              % (f16, PEAK_FP16_TFLOPS, f32, PEAK_FP32_TFLOPS),
                "vs_fp32_mfma_peak": round(achieved / PEAK_FP32_TFLOPS, 4)}
    if name == "nfk_fused_realnvp":
        H, n = kw["hidden_dim"], kw["dim"] // 2
        kbf, R = divmod(H, 32)
        tail = R if (0 < R <= 4 and kbf >= 1) else 0
        f32 = 4 * 2.0 * tail * (H + n)                       # k-tails of layers 2-3, 4 nets
        f16 = 4 * 2.0 * (n * H + H * H + H * n) - f32         # 131,200/sample
        flops = (f16 + f32) * B
        t_floor = f32 / (PEAK_FP32_TFLOPS * 1e12) + 3.0 * f16 / (PEAK_FP16_TFLOPS * 1e12)
        peak = (f16 + f32) / t_floor / 1e12
        achieved = flops / (mean_ms * 1e-3) / 1e12
        return {"kernel": name, "bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 1),
                "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
                "launches": n_launch, "mean_ms": round(mean_ms, 4),
                "per_launch": "%d samples x %.0f flop (fp32-equivalent)" % (B, flops / B),
                "peak_basis": "MFMA floor: %.0f flop/sample as 3 fp16 products + %.0f on f32 MFMA"
                              % (f16, f32)}
    if name == "nfk_rqs_coupling":
        n_up = kw["size"] * (kw["dim"] - 1)
        P = 3 * kw["K"] - 1
        byts = (D * 4 + n_up * P * 4 + D * 4 + 8) * B            # 3,464 B/sample
    elif name == "nfk_affine_coupling":
        n = D // 2
        byts = (n * 4 * 2 + n * 4 * 2 + 8) * B                   # x half r/w + s,t + logdet RMW
    elif name == "nfk_normal_logprob":
        byts = (D * 4 + 4 + 4) * B
    else:
        return None
    achieved = byts / (mean_ms * 1e-3) / 1e9
    return {"kernel": name, "bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
            "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
            "launches": n, "mean_ms": round(mean_ms, 4),
            "per_launch": "%d samples x %.0f B" % (B, byts / B)}


def load_traffic(kernel, workload):
    """HBM bytes per launch from a committed rocprofv3 PMC summary, if any
    (profiles/pmc_traffic.json: entries keyed "<workload>:<kernel>", or by the
    kernel alone for the c3 default)."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            tab = json.load(f)
    except (OSError, ValueError):
        return None
    rec = tab.get("%s:%s" % (workload, kernel))
    if rec is None and workload == "c3":
        rec = tab.get(kernel)
    return None if rec is None else rec.get("bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=1 << 20, help="samples per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timer", action="store_true", help="skip the per-kernel event timer")
    ap.add_argument("--unfused", action="store_true", help="disable the fused MFMA layer kernel")
    ap.add_argument("--no-chain", action="store_true",
                    help="one fused launch per layer instead of one chained launch per run of layers")
    args = ap.parse_args()

    from normalizingflow_amd import config, dist as nfdist, kernels
    import torch.distributed as dist

    rank, world, local = nfdist.init_from_env()
    if world != args.gpus and rank == 0:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    config.USE_FUSED = not args.unfused
    config.USE_CHAIN = not args.no_chain

    model, sd, _ = build_model(args.workload, device)
    B = args.batch
    D = WORKLOADS[args.workload][3]
    g = torch.Generator(device=device).manual_seed(rank)
    x = torch.randn(B, D, generator=g, device=device)  # resident in HBM before timing

    def step():
        lp = model.log_prob(x)
        if world > 1:
            nfdist.nll_allreduce(lp)
        return lp

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    timer = None
    if not args.no_timer:
        timer = kernels.TIMER = kernels.KernelTimer()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    kernels.TIMER = None
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    summary = timer.summary() if timer is not None else {}

    if rank == 0:
        value = world * B * args.steps / dt
        dom = max(summary.items(), key=lambda kv: kv[1][2])[0] if summary else None
        rl = roofline(args.workload, summary, B, load_traffic(dom, args.workload) if dom else None,
                      args.steps)
        cpu = None
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline is an N=1 figure
            cpu = cpu_baseline(args.workload, {k: v.cpu() for k, v in sd.items()})
        desc = WORKLOADS[args.workload][0]
        out = {
            "metric": METRICS[args.workload],
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic x ~ N(0, I) resident in HBM; random-init weights (seed 1234)",
            "config": {"workload": args.workload + ": " + desc, "global_batch": world * B,
                       "per_gpu_batch": B, "parallelism": "dp%d (sample sharding)" % world,
                       "fused_layer_kernel": bool(config.USE_FUSED),
                       "chained_layers": bool(config.USE_FUSED and config.USE_CHAIN),
                       "conditioner_arith": ARITH.get(args.workload) if config.USE_FUSED
                       else "f32 (rocBLAS)"},
            "roofline": rl,
            "cpu_baseline": cpu,
            "kernels": {k: {"launches": v[0], "mean_ms": round(v[1], 4)} for k, v in summary.items()},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
