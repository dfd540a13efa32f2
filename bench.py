#!/usr/bin/env python
"""Throughput of the log_prob hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c5|c1]
                    [--scaling weak|strong] [--batch B] [--global-batch G]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

``--gpus N`` alone (no launcher, WORLD_SIZE unset) starts the N rank
processes itself (spawn_ranks: torchrun's environment, one per GPU).

A step = one NormalizingFlowModel.log_prob pass over this rank's rows of
synthetic x ~ N(0, I), already resident in HBM (c3: 8 NSF_CL RQS coupling
layers, D=64, K=8, H=100).  Sample sharding, replicated weights:
  --scaling weak   (default at N = 1) every rank owns --batch rows (2^20):
                   BASELINE config c4 (8M rows over 8 GPUs);
  --scaling strong the --global-batch rows (2^20) are split over the ranks
                   (dist.shard_range): the north star's strong-scaling target;
  --scaling both   (default at N > 1) both loops in one invocation: weak is
                   the line's value, strong is its "strong" sub-object.
With N > 1 each step ends with the NLL all-reduce of [sum log p, count]
(RCCL; --backend gloo runs the same path over gloo, e.g. N ranks on one
device in a test).  Status checks run deferred (config.STRICT_CHECKS =
"deferred": no host sync per step; flushed, and raised, after the timed loop).

Rank 0 prints ONE JSON line with:
  roofline      the dominant kernel's time from HIP events recorded live on
                its launch stream, against a hardware roofline: the dense
                f16 MFMA peak for the fused kernels (frac = the MFMA floor of
                the kernel's formulation / the launch time), HBM for the
                streaming ones (and for the fused NSF_AR at batches where
                reading its weights once is the larger floor); the VALU-issue
                floor from the committed PMC instruction counts
                (profiles/pmc_insts.json) is a diagnostic entry of `floors`;
                traffic = PMC HBM bytes per launch
  parity        the oracle's log_prob on the first --parity-rows rows of the
                benched x and weights vs the values the timed kernel produced
                (outside the timed region)
  cpu_baseline  the CPU oracle (torch-CPU fp32 restatement of the reference
                path) on a bounded sample of the same workload, best of 3
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
    # BASELINE c1 (the reference's CPU-runnable case) on the GPU: the D = 2
    # halves run zero-padded to the fused RealNVP chain's half-dimension 16
    # (RealNVP._fused_half); 4096 rows are launch- and latency-bound
    "c1": ("2-D two moons (noise 0.05, seed 0), 4-layer RealNVP affine coupling (H=100), log_prob",
           "RealNVP", dict(dim=2, hidden_dim=100), 2, 4),
    # the applications' default flow type (config.py:37) at applications/input/
    # Gaussian.yaml's shape: 20 particles x 2 dims, nsplines 10, hidden 80,
    # nlayers 1, B = ncellx * cell_len / 2 = 4 (setup.py:42, 58)
    "ar": ("40-dim synthetic Gaussian, NSF_AR autoregressive RQS (Gaussian.yaml: K=10, H=80, B=4, "
           "1 layer), log_prob", "NSF_AR", dict(dim=40, K=10, B=4.0, hidden_dim=80), 40, 1),
    # the applications' own NSF_AR (Einstein.yaml; LJ.yaml and Fe_*.yaml share the
    # flow): 32 particles x 3 dims, nsplines 32, hidden 354, nlayers 2,
    # B = (nparticles / (8 rho))^(1/3) at rho 1.28 (setup.py:42-58)
    "ar354": ("96-dim synthetic Gaussian, NSF_AR autoregressive RQS (Einstein.yaml: K=32, H=354, "
              "B=1.462, 2 layers), log_prob", "NSF_AR",
              dict(dim=96, K=32, B=(32 / (8 * 1.28)) ** (1.0 / 3.0), hidden_dim=354), 96, 2),
    # the Fe configs' flow (applications/input/Fe_100K.yaml; Fe_400K / Fe_700K the
    # same): 54 particles x 3 dims = 162 coordinates, nsplines 32, hidden 354,
    # nlayers 2, B = ncellx * cell_len / 2 = 3 * 2.8841 / 2 (setup.py:44-58)
    "fe162": ("162-dim synthetic Gaussian, NSF_AR autoregressive RQS (Fe_*.yaml: K=32, H=354, "
              "B=4.326, 2 layers), log_prob", "NSF_AR", dict(dim=162, K=32, B=3 * 2.8841 / 2, hidden_dim=354),
              162, 2),
    # Polymer.yaml's flow: 2048 particles x 1 dim, nsplines 32, hidden_dim from
    # config.py:40 (100), nlayers 2, B = ncellx * cell_len / 2 = 0.5
    "poly2048": ("2048-dim synthetic Gaussian, NSF_AR autoregressive RQS (Polymer.yaml: K=32, H=100, "
                 "B=0.5, 2 layers), log_prob", "NSF_AR", dict(dim=2048, K=32, B=0.5, hidden_dim=100), 2048, 2),
    # Polymer_rnvp.yaml's flow, the config the reference's Polymer driver loads
    # (applications/examples/polymer.py:29): RealNVP(2048, hidden 4000) x 10,
    # batch 40 (:30); each layer is its 387 MB of weights at these batches
    "rnvp2048": ("2048-dim synthetic Gaussian, 10-layer RealNVP affine coupling (Polymer_rnvp.yaml: H=4000), "
                 "log_prob", "RealNVP", dict(dim=2048, hidden_dim=4000), 2048, 10),
}
# default per-GPU rows: c1 is BASELINE's 4,096-row case; ar354 runs at its
# configs' own training batch (Einstein.yaml / LJ.yaml batch_size 40), where
# the fused layer splits its conditioners over the GPU (nfk_fused_ar_ws)
DEFAULT_BATCH = {"c1": 4096, "ar354": 40, "fe162": 50, "poly2048": 40, "rnvp2048": 40}
# BASELINE.md's figures for the same metric and config: the reference's own
# CPU path measured in the survey container (8-core Xeon, 8 threads, fp32;
# no GPU figures exist): c1 at B = 4096, c2 and c3 at B = 2^20 (c5 is quoted
# there at B = 65,536 only, so it has none here)
BASELINE_CPU = {"c1": 900334.0, "c2": 126376.0, "c3": 13918.0}


def moons(n, noise=0.05, generator=None, device="cpu"):
    """Two interleaved half circles (the sklearn make_moons formula, SURVEY
    8(d) c1: noise 0.05, seed 0): n // 2 points on the outer arc, the rest on
    the inner one, shuffled, plus N(0, noise^2) jitter."""
    n_out = n // 2
    n_in = n - n_out
    t_out = torch.linspace(0, torch.pi, n_out, dtype=torch.float64)
    t_in = torch.linspace(0, torch.pi, n_in, dtype=torch.float64)
    x = torch.cat([torch.stack([torch.cos(t_out), torch.sin(t_out)], 1),
                   torch.stack([1 - torch.cos(t_in), 1 - torch.sin(t_in) - 0.5], 1)]).float()
    gd = generator.device if generator is not None else torch.device("cpu")
    perm = torch.randperm(n, generator=generator, device=gd).cpu()
    x = x[perm] + noise * torch.randn(n, 2, generator=generator, device=gd).cpu()
    return x.to(device)


def make_x(workload, n, generator, device):
    """The workload's synthetic rows: two moons for c1, x ~ N(0, I) otherwise."""
    if workload == "c1":
        return moons(n, generator=generator, device=device)
    return torch.randn(n, WORKLOADS[workload][3], generator=generator, device=device)


METRICS = {
    "c3": "samples/sec log_prob (1M×64, 8 RQS coupling layers) at 1/2/4/8 GPU",  # BASELINE.json
    "c2": "samples/sec log_prob (1M×64, 8 RealNVP affine coupling layers)",
    "c5": "samples/sec log_prob (1M×256, 16 RQS coupling layers, H=256, K=16)",
    "c1": "samples/sec log_prob (4096×2 two moons, 4 RealNVP affine coupling layers)",
    "ar": "samples/sec log_prob (1M×40, 1 NSF_AR autoregressive RQS layer, K=10, H=80)",
    "ar354": "samples/sec log_prob (96-dim rows, 2 NSF_AR autoregressive RQS layers, K=32, H=354; rows per step = config.global_batch, default the applications' 40)",
    "fe162": "samples/sec log_prob (162-dim rows, 2 NSF_AR autoregressive RQS layers, K=32, H=354; rows per step = config.global_batch, default the Fe configs' 50)",
    "poly2048": "samples/sec log_prob (2048-dim rows, 2 NSF_AR autoregressive RQS layers, K=32, H=100; rows per step = config.global_batch, default Polymer.yaml's 40)",
    "rnvp2048": "samples/sec log_prob (2048-dim rows, 10 RealNVP affine coupling layers, H=4000; rows per step = config.global_batch, default Polymer_rnvp.yaml's 40)",
}


# conditioner arithmetic of the fused layer kernels per workload
_SPLIT = "fp16 two-way split (hi+lo, 3 MFMA products, fp32 accumulate, power-of-two pre-scaling)"
_TAIL = "; the 4 tail features of H=100 as one 16x16x16 f16 MFMA per tile holding the same 3 products"
ARITH = {
    "c3": _SPLIT + _TAIL + " (nfk_fused_impl.h)",
    "c2": _SPLIT + _TAIL + " (nfk_fused_rnvp.hip)",
    "c5": _SPLIT + " (nfk_fused_wide.h)",
    "c1": _SPLIT + _TAIL + " (nfk_fused_rnvp.hip; the D = 2 halves zero-padded to the kernel's 16)",
    "ar": _SPLIT + " (nfk_fused_ar.hip; layer 1 on the fp16-split trig features)",
    "ar354": _SPLIT + "; the 2 tail features of H=354 as one 16x16x16 f16 MFMA per tile"
             " (nfk_fused_ar.hip, one wave per SIMD; layer 1 on the fp16-split trig features)",
    "fe162": _SPLIT + "; the 2 tail features of H=354 as one 16x16x16 f16 MFMA per tile"
             " (nfk_fused_ar.hip, one wave per SIMD; layer 1 on the fp16-split trig features)",
    "poly2048": _SPLIT + _TAIL + " (nfk_fused_ar.hip; layer 1 on the fp16-split trig features)",
    "rnvp2048": _SPLIT + " (nfk_wide_rnvp.hip: weight-stream GEMMs, the hidden layers' GEMM + tanh fused up to 64 rows, the output layer split-K with fp32 partial sums added in split order; the 10 layers in one nfk_wide_rnvp_chain call)",
}
# the line's dtype: what the path computes in (fp32 values and outputs; the
# conditioner's products on the fp16 matrix cores as a two-way split)
DTYPE_FUSED = "fp32 (conditioner GEMMs: 3x fp16-split MFMA, fp32 accumulate; spline fp32)"
PARITY_RTOL = 1e-5   # BASELINE.json north star: log_prob within 1e-5 relative (fp32)
PARITY_ATOL = 1e-5   # ... with this absolute floor for values near 0 (tests/test_gpu_parity.py)
CLOCK_GHZ = 2.4      # MI355X_MICROARCH.md: max engine clock
N_SIMD = 1024        # 256 CUs x 4 SIMDs
# VALU issue cost per wave64 instruction on one SIMD with several waves
# resident, calibrated on wall-clock time (tools/ubench_valu.hip,
# profiles/r2_ubench_valu.txt: at 2-4 waves per SIMD one v_add_f32 / v_fma_f32
# takes 1.77-2.02 ns of the SIMD, one v_exp_f32 3.48-3.56 ns, i.e. 4.2-4.9 and
# 8.4-8.6 cycles at 2.4 GHz -- MI355X_MICROARCH.md's issue table says 4 and 8),
# and MI355X_MICROARCH.md: an MFMA holds the SIMD's vector issue for 8 cycles.
# (Rounds 2-4 used 2 and 4, read off the per-wave s_memtime column; the
# wall-clock figures are what a launch pays.)
VALU_CYC, TRANS_CYC, MFMA_HOLD_CYC = 4.4, 8.4, 8.0


def build_model(workload, device):
    import nf.flows as nff
    import nf.models as nfm
    desc, kind, kw, D, L = WORKLOADS[workload]
    torch.manual_seed(1234)  # weights seed 1234, nn.Linear default init, on CPU
    if kind == "NSF_CL":
        flows = [nff.NSF_CL(mask=[i % 2], **kw) for i in range(L)]
    elif kind == "NSF_AR":
        flows = [nff.NSF_AR(**kw) for _ in range(L)]
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
    if kind == "NSF_AR":
        return [dict(type="NSF_AR", prefix="flows.%d." % i, dim=kw["dim"], K=kw["K"], B=kw["B"])
                for i in range(L)]
    return orc.realnvp_specs(L, kw["dim"])


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


_T0 = time.perf_counter()


def progress(msg):
    """A timestamped progress line on stderr (long GPU-box runs must keep writing)."""
    print("[bench %7.1fs] %s" % (time.perf_counter() - _T0, msg), file=sys.stderr, flush=True)


def cgroup_cpus():
    """The job's CPU quota in whole CPUs from cgroup v2 cpu.max (v1's
    cfs_quota / cfs_period), or None when unlimited / unreadable."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as f:
                txt = f.read().strip()
            if parse is not None:
                q, per = parse(txt)
                if q == "max":
                    return None
                return max(1, int(int(q) // int(per)))
            q = int(txt)
            if q <= 0:
                return None
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                return max(1, q // int(f.read().strip()))
        except (OSError, ValueError):
            continue
    return None


def host_cores():
    """CPUs this job may use: the affinity mask, capped by the cgroup CPU
    quota (os.cpu_count() on the GPU box counts the whole machine's 256, of
    which a one-GPU job gets a 16-CPU share: 256 threads on it thrash)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q = cgroup_cpus()
    return min(n, q) if q else n


def cpu_baseline(workload, sd, budget_s=12.0):
    """BASELINE.md's CPU-baseline plan: the CPU oracle on all host cores and
    at the job's thread share (OMP_NUM_THREADS, 16 on the GPU box), each on a
    bounded sample (about budget_s of CPU work); the reported value is the
    faster of the two (the better CPU baseline), both are in the record."""
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or torch.get_num_threads()
    allc = host_cores()
    skipped = None
    settings = {share, allc}
    if cgroup_cpus() is None and allc > 2 * share:
        # no readable quota and far more CPUs in the mask than the job's thread
        # share (the one-GPU box: 256 vs 16): a 256-thread run measured > 170 s
        # for one 4096-row warm-up there (thrashing), so only the share is timed
        settings = {share}
        skipped = "%d threads (affinity mask) not timed: no cgroup quota readable and the job's " \
                  "share is OMP_NUM_THREADS=%d" % (allc, share)
    prev = torch.get_num_threads()
    runs = {}
    try:
        for n in sorted(settings):
            torch.set_num_threads(n)
            progress("cpu baseline: %d threads" % n)
            runs[n] = _cpu_baseline_at(workload, sd, budget_s)
            progress("cpu baseline: %d threads -> %.1f samples/s" % (n, runs[n]["value"]))
    finally:
        torch.set_num_threads(prev)
    best = max(runs.values(), key=lambda r: r["value"])
    out = dict(best)
    out["by_threads"] = {str(n): {"value": round(r["value"], 1), "runs_s": r["runs_s"]}
                         for n, r in runs.items()}
    out["all_host_cores"] = allc
    out["thread_share"] = share
    out["cgroup_cpus"] = cgroup_cpus()
    out["skipped"] = skipped
    out["affinity_cpus"] = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return out


def _cpu_baseline_at(workload, sd, budget_s):
    """The oracle at the current torch thread count: warm-ups that size the
    sample, then the best of 3 timed runs.  A workload quoted at a small batch
    (c1: 4096 rows) is timed as repeated passes over one batch of that size."""
    from oracle import nf_oracle as orc
    D = WORKLOADS[workload][3]
    specs = specs_for(workload)
    g = torch.Generator().manual_seed(0)
    small = DEFAULT_BATCH.get(workload)
    with torch.inference_mode():
        x = make_x(workload, small or 4096, g, "cpu")
        for _ in range(2):  # the first call pays one-time setup; the second gives the rate
            t0 = time.perf_counter()
            orc.model_log_prob(specs, sd, x)
            t_w = time.perf_counter() - t0
        reps = 1
        if small:
            reps = int(max(1, (budget_s / 3) / max(t_w, 1e-4)))
            n = small
        else:
            n = int(max(4096, min(1 << 20, 4096 * (budget_s / 3) / max(t_w, 1e-3))))
            n = (n // 4096) * 4096
            x = make_x(workload, n, g, "cpu")
        runs = []
        for _ in range(3):
            t0 = time.perf_counter()
            for _ in range(reps):
                orc.model_log_prob(specs, sd, x)
            runs.append(time.perf_counter() - t0)
            progress("cpu baseline run: %d x %d rows in %.2f s" % (reps, n, runs[-1]))
    dt = min(runs)
    return {"value": n * reps / dt, "unit": "samples/s", "cores": torch.get_num_threads(),
            "kind": "port", "nproc": os.cpu_count(), "cpu_model": _cpu_model(),
            "runs_s": [round(r, 3) for r in runs],
            "sample": "%s log_prob of %d x %d x %d rows (seed 0) by the CPU oracle (oracle/nf_oracle.py: "
                      "torch-CPU fp32 restatement of nf/models.py:37 evaluate), %d threads, "
                      "2 warm-ups + best of 3 timed runs (%.1f s best)"
                      % (workload, reps, n, D, torch.get_num_threads(), dt)}


def parity(workload, sd, x_rows, lp_rows):
    """The oracle on the first rows of the benched x (same weights) vs the
    log_prob the benched kernel produced for them."""
    from oracle import nf_oracle as orc
    with torch.inference_mode():
        ref = orc.model_log_prob(specs_for(workload), sd, x_rows)
    d = (lp_rows.double() - ref.double()).abs()
    rel = d / ref.double().abs().clamp_min(1e-30)
    ok = bool((d <= PARITY_ATOL + PARITY_RTOL * ref.double().abs()).all())
    return {"rows": int(x_rows.shape[0]), "max_rel_dlog_prob": float(rel.max()),
            "max_abs_dlog_prob": float(d.max()), "rtol": PARITY_RTOL, "atol": PARITY_ATOL,
            "pass": ok, "reference": "oracle/nf_oracle.py model_log_prob (pinned by tests/golden)"}


def load_insts(kernel, workload):
    """Per-launch PMC instruction counts of the kernel (profiles/pmc_insts.json,
    entries "<workload>:<kernel>"), or None."""
    try:
        with open(os.path.join(REPO, "profiles", "pmc_insts.json")) as f:
            return json.load(f).get("%s:%s" % (workload, kernel))
    except (OSError, ValueError):
        return None


def valu_floor_ms(insts, per_launch_scale=1.0):
    """VALU-issue floor of one launch: every SIMD's vector issue port busy for
    the launch's VALU instructions (transcendentals at their higher cost) and
    the cycles each MFMA holds it, spread over the 1024 SIMDs at the max clock."""
    if not insts:
        return None
    # (SQ_INSTS_VALU counts the MFMAs too: they are priced by their issue hold only)
    cyc = (VALU_CYC * (insts["valu"] - insts["valu_trans"] - insts["mfma"]) + TRANS_CYC * insts["valu_trans"]
           + MFMA_HOLD_CYC * insts["mfma"]) * per_launch_scale
    return cyc / N_SIMD / (CLOCK_GHZ * 1e9) * 1e3


MFMA_CYC = 16.0  # MI355X_MICROARCH.md: 16x16x32 f16/bf16 back-to-back on one SIMD (16x16x16 f16 the same)


def mfma_per_wave_layer(workload):
    """MFMA instructions one 16-sample wave issues per layer in the fused
    kernels' formulation: per (output tile, 32-wide k-block) the 3 fp16-split
    products, per tile one tail MFMA when H = 32 KBH + 1..4."""
    desc, kind, kw, D, L = WORKLOADS[workload]
    H = kw["hidden_dim"]
    kbf, R = divmod(H, 32)
    T1 = 1 if (0 < R <= 4 and kbf >= 1) else 0
    KBH = kbf if (R == 0 or T1) else kbf + 1
    HT = 2 * KBH + T1
    per_tile = 3 * KBH + T1
    if kind == "RealNVP":
        n = (kw["dim"] // 2 + 15) // 16 * 16  # the kernel's half-dimension (c1's D = 2 runs padded to 16)
        NO, KBI = n // 16, (n // 16 + 1) // 2
        return 4 * (KBI * HT * 3 + HT * per_tile + NO * per_tile)
    n_lo, n_up = kw["size"], kw["size"] * (kw["dim"] - 1)
    K = kw["K"]
    if n_lo + n_up <= 128:  # k_fused_nsf: 16-coordinate chunks of W, H (K tiles), D (K-1)
        tiles = ((n_up + 15) // 16) * (3 * K - 1)
    else:                   # k_fused_nsf_wide: 8-coordinate chunks of ceil(K/2), ceil(K/2), K/2 tiles
        tiles = ((n_up + 7) // 8) * (2 * ((K + 1) // 2) + K // 2)
    return ((n_lo + 31) // 32) * HT * 3 + HT * per_tile + tiles * per_tile


# dense f16 MFMA peak: one 16x16x32 f16 MFMA (16,384 flop) per 16 cycles per
# SIMD on 1024 SIMDs at 2.4 GHz = 2,516.6 TFLOP/s (MI355X_MICROARCH.md; AMD's
# 2:1-sparsity figure is not used)
MFMA_FLOP = 2 * 16 * 16 * 32
PEAK_MFMA_F16_TFLOPS = MFMA_FLOP / 16.0 * 1024 * 2.4e9 / 1e12


def _floors(B, per, insts, n_mfma):
    """(t_mfma_ms, floors) of a fused kernel launch: the MFMA floor of its
    formulation (n_mfma instructions per 16 samples and layer at MFMA_CYC
    each on the 1024 SIMDs: the hardware roofline) and, as a diagnostic when
    its PMC instruction counts are committed, the VALU-issue floor."""
    t_mfma = n_mfma * MFMA_CYC * (B / 16.0) * per / N_SIMD / (CLOCK_GHZ * 1e9) * 1e3
    floors = {"mfma_ms": round(t_mfma, 4),
              "mfma_basis": "%d MFMA per 16 samples and layer x %g cyc on 1024 SIMDs at %.1f GHz"
                            % (n_mfma, MFMA_CYC, CLOCK_GHZ)}
    if insts:
        scale = (B / insts["batch"]) * (per / insts.get("layers", 1))
        floors["valu_issue_ms"] = round(valu_floor_ms(insts, scale), 4)
        floors["valu_basis"] = ("diagnostic, not the roofline: %.0f VALU (%.0f transcendental) + %.0f MFMA "
                                "per launch of %d samples x %g layers (%s); %g cyc per VALU, %g per "
                                "transcendental, %g per MFMA issue hold, on 1024 SIMDs at %.1f GHz"
                                % (insts["valu"], insts["valu_trans"], insts["mfma"], insts["batch"],
                                   insts.get("layers", 1), insts.get("source", "PMC"), VALU_CYC,
                                   TRANS_CYC, MFMA_HOLD_CYC, CLOCK_GHZ))
    return t_mfma, floors


def _mfma_roofline(name, n_mfma, B, per, mean_ms, t_mfma, ref_flops, floors):
    """The MFMA-bound roofline fields: achieved = the MFMA pipe's work of the
    launch (its n_mfma instructions per 16 samples and layer, each one
    16x16x32-f16 issue slot = 16,384 flop) / the launch time, peak = the dense
    f16 MFMA peak, so frac = the MFMA floor / the launch time."""
    mflops = n_mfma * MFMA_FLOP * (B / 16.0) * per
    achieved = mflops / (mean_ms * 1e-3) / 1e12
    if "valu_issue_ms" in floors:  # the binding pipe of the VALU-heavy formulations (diagnostic)
        floors["valu_issue_frac"] = round(floors["valu_issue_ms"] / mean_ms, 4)
    return {"kernel": name, "bound": "mfma", "achieved": round(achieved, 2),
            "peak": round(PEAK_MFMA_F16_TFLOPS, 1), "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_MFMA_F16_TFLOPS, 4),
            "mfma_frac": round(t_mfma / mean_ms, 4),
            "floor_ms": round(t_mfma, 4), "floors": floors,
            "peak_basis": "dense f16 MFMA peak (16x16x32 f16: 16,384 flop per 16 cycles per SIMD, 1024 SIMDs, "
                          "2.4 GHz); achieved = the launch's MFMA issue slots x 16,384 flop / launch time "
                          "(the 16x16x16 tail MFMAs occupy a full slot)",
            "ref_fp32_equiv_tflops": round(ref_flops / (mean_ms * 1e-3) / 1e12, 2),
            "ref_fp32_equiv_basis": "the reference FCNN's fp32 flops (SURVEY 8(d)) / launch time",
            "vs_fp32_mfma_peak": round(ref_flops / (mean_ms * 1e-3) / 1e12 / PEAK_FP32_TFLOPS, 4)}


def roofline(workload, timer_summary, per_gpu_batch, traffic, n_steps):
    """Roofline of the dominant kernel from live HIP-event timings, against
    the kernel's binding floor (see _floors)."""
    if not timer_summary:
        return None
    name, (n_launch, mean_ms, tot) = max(timer_summary.items(), key=lambda kv: kv[1][2])
    desc, kind, kw, D, L = WORKLOADS[workload]
    B = per_gpu_batch
    insts = load_insts(name, workload)
    if name in ("nfk_fused_nsf", "nfk_fused_nsf_chain", "nfk_fused_realnvp", "nfk_fused_realnvp_chain"):
        H = kw["hidden_dim"]
        kbf, R = divmod(H, 32)
        tail = R if (0 < R <= 4 and kbf >= 1) else 0
        if name in ("nfk_fused_realnvp", "nfk_fused_realnvp_chain"):
            per = L * n_steps / n_launch if name == "nfk_fused_realnvp_chain" else 1
            n = kw["dim"] // 2
            f32 = 4 * 2.0 * tail * (H + n)                       # k-tails of layers 2-3, 4 nets
            f16 = 4 * 2.0 * (n * H + H * H + H * n) - f32         # 131,200/sample
        else:
            # layers per launch: all L of a step in one chain launch (or one per launch)
            per = L * n_steps / n_launch if name == "nfk_fused_nsf_chain" else 1
            n_lo = kw["size"]  # mask of one coordinate per particle (dim=2)
            n_up = kw["size"] * (kw["dim"] - 1)
            P = 3 * kw["K"] - 1
            f32 = 2.0 * tail * (H + n_up * P)
            f16 = 2.0 * (n_lo * H + H * H + H * n_up * P) - f32  # 173,600/sample/layer
        flops = (f16 + f32) * B * per
        n_mfma = mfma_per_wave_layer(workload)
        t_mfma, floors = _floors(B, per, insts, n_mfma)
        alg = (D * 4 + 4) * B if name.endswith("_chain") else (2 * D * 4 + 8) * B  # x (+ z, log|det|) or log p
        out = _mfma_roofline(name, n_mfma, B, per, mean_ms, t_mfma, flops, floors)
        out.update({"traffic": traffic, **hbm_fields(traffic, alg, mean_ms),
                    "launches": n_launch, "mean_ms": round(mean_ms, 4),
                    "per_launch": "%d samples x %g layers: %d MFMA per 16 samples and layer; reference "
                                  "%.0f flop per sample and layer (fp32-equivalent)"
                                  % (B, per, n_mfma, flops / B / per)})
        return out
    if name == "nfk_fused_ar":
        return roofline_ar(kw, B, L * n_steps / n_launch, n_launch, mean_ms, traffic, insts)
    if name in ("nfk_wide_rnvp", "nfk_wide_rnvp_chain"):
        # nl layers per launch (the chain: the model's whole run of them), each
        # layer's four FCNNs' weights read once (fp16 hi + lo: 4 B per weight,
        # the fp32 bytes) + x in, z out, log|det| RMW
        nl = max(1, int(round(L * n_steps / n_launch)))
        D2, H = kw["dim"] // 2, kw["hidden_dim"]
        wts = 4 * 4 * (D2 * H + H + H * H + H + H * D2 + D2)
        byts = nl * wts + (2 * kw["dim"] * 4 + 8) * B
        achieved = byts / (mean_ms * 1e-3) / 1e9
        return {"kernel": name, "bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                **hbm_fields(traffic, byts, mean_ms), "launches": n_launch, "mean_ms": round(mean_ms, 4),
                "floor_ms": round(byts / (PEAK_HBM_GBS * 1e9) * 1e3, 4),
                "per_launch": "%d samples x %d layer(s): %d B algorithmic (each layer's weights once + x, z, "
                              "log|det|; streamed once per 128-row pass)" % (B, nl, byts)}
    if name == "nfk_rqs_coupling" and kind == "NSF_AR":
        P = 3 * kw["K"] - 1
        byts = (4 + P * 4 + 4 + 8) * B                            # one column: x, params, z, log|det| RMW
    elif name == "nfk_rqs_coupling":
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
            **hbm_fields(traffic, byts, mean_ms),
            "launches": n_launch, "mean_ms": round(mean_ms, 4),
            "per_launch": "%d samples x %.0f B" % (B, byts / B)}


def hbm_fields(traffic, alg_bytes, mean_ms):
    """The launch against the HBM roofline: algorithmic bytes and, when a PMC
    summary is committed, the measured HBM bytes (traffic), each / the
    launch time, as GB/s and as a fraction of the 8 TB/s peak."""
    t = mean_ms * 1e-3
    out = {"alg_hbm_bytes": int(alg_bytes), "alg_hbm_gbs": round(alg_bytes / t / 1e9, 1),
           "alg_hbm_frac": round(alg_bytes / t / 1e9 / PEAK_HBM_GBS, 4),
           "hbm_gbs": None, "hbm_frac": None}
    if traffic:
        out["hbm_gbs"] = round(traffic / t / 1e9, 1)
        out["hbm_frac"] = round(traffic / t / 1e9 / PEAK_HBM_GBS, 4)
    return out


def ar_weight_bytes(dim, K, H):
    """Bytes of one NSF_AR layer's conditioner weights and biases at 4 B each
    (FCNN(2i, 3K-1, H), i = 1 .. dim-1, flows.py:166-167)."""
    P = 3 * K - 1
    return 4 * sum(2 * i * H + H + H * H + H + P * H + P for i in range(1, dim))


def ar_mfma_per_wave_layer(dim, K, H):
    """MFMA instructions of one 16-sample wave per NSF_AR layer in
    nfk_fused_ar's formulation: conditioner i = 1 .. dim-1 runs layer 1 over
    ceil(2i / 32) k-blocks and HT hidden tiles (3 split products each), layer 2
    and the output layer (ceil((3K-1) / 16) tiles) over KBH k-blocks (+1 tail
    MFMA per tile when H = 32 KBH + 1..4, +2 when H = 32 KBH + 5..16: the
    16-feature half tile, nfk_fused_ar.hip ar_dims)."""
    kbf, R = divmod(H, 32)
    TK = 0 if (R == 0 or kbf < 1) else (1 if R <= 4 else (2 if R <= 16 else 0))
    KBH = kbf if (R == 0 or TK) else kbf + 1
    HT, NO = 2 * KBH + (1 if TK else 0), (3 * K - 1 + 15) // 16
    per_tile = 3 * KBH + TK
    return sum(((2 * i + 31) // 32) * HT * 3 + (HT + NO) * per_tile for i in range(1, dim))


def roofline_ar(kw, B, per, n_launch, mean_ms, traffic, insts):
    """nfk_fused_ar: the reference's FCNN flops of every conditioner
    (sum_i 2 (2i H + H H + H (3K-1)) per sample) against the binding floor of
    the kernel's formulation (MFMA; VALU issue when PMC counts are committed)."""
    dim, K, H = kw["dim"], kw["K"], kw["hidden_dim"]
    fl = sum(2.0 * (2 * i * H + H * H + H * (3 * K - 1)) for i in range(1, dim))
    flops = fl * B * per
    n_mfma = ar_mfma_per_wave_layer(dim, K, H)
    t_mfma, floors = _floors(B, per, insts, n_mfma)
    # x in, z and log|det| out, and every conditioner's weights once per launch
    # (fp16 hi + lo: 4 B per weight; a launch must read them at least once)
    alg = ((2 * dim * 4 + 8) * B + ar_weight_bytes(dim, K, H)) * per
    # at small batches the weights dominate: reading them once at the HBM peak
    # is then the binding floor (the applications' 40 rows: 73.6 MB per launch)
    t_hbm = alg / (PEAK_HBM_GBS * 1e9) * 1e3
    floors["hbm_ms"] = round(t_hbm, 4)
    if t_hbm > t_mfma:
        achieved = alg / (mean_ms * 1e-3) / 1e9
        return {"kernel": "nfk_fused_ar", "bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4), "mfma_frac": round(t_mfma / mean_ms, 4),
                "traffic": traffic,
                **hbm_fields(traffic, alg, mean_ms), "launches": n_launch, "mean_ms": round(mean_ms, 4),
                "floor_ms": round(t_hbm, 4), "floors": floors,
                "per_launch": "%d samples x %g layers: %d B algorithmic (weights once + x, z, log|det|)"
                              % (B, per, alg)}
    out = _mfma_roofline("nfk_fused_ar", n_mfma, B, per, mean_ms, t_mfma, flops, floors)
    out.update({"traffic": traffic, **hbm_fields(traffic, alg, mean_ms), "launches": n_launch,
                "mean_ms": round(mean_ms, 4),
                "per_launch": "%d samples x %g layers: %d MFMA per 16 samples and layer; reference %.0f flop "
                              "per sample and layer (FCNN flops, fp32-equivalent)" % (B, per, n_mfma, fl)})
    return out


def load_traffic(kernel, workload, batch=None):
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
    if rec is None or not rec.get("bytes_per_launch"):
        return None
    # an entry measured at another batch is scaled to this one (streaming
    # kernels: bytes per row), unless its bytes do not scale with the batch
    # (the fused NSF_AR's weight stream: "batch_exact")
    if rec.get("batch_exact") and batch is not None and batch != rec.get("batch"):
        return None
    scale = 1.0 if batch is None else batch / float(rec.get("batch", 1 << 20))
    return int(rec["bytes_per_launch"] * scale)


def spawn_ranks(n):
    """``--gpus N`` (N > 1) started without a launcher (no WORLD_SIZE in the
    environment): start the N rank processes of this same command line, one
    per GPU, with torchrun's environment contract (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT), before anything in
    this process touches the GPU (child processes, no exec).  Rank 0 prints the
    line.  If a rank fails the others are stopped (by their own PIDs) and its
    exit code is returned."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        time.sleep(0.2)
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for o in procs:  # a failed rank leaves the others waiting on a collective
                    o.kill()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--scaling", default=None, choices=("weak", "strong", "both"),
                    help="weak: --batch rows per GPU; strong: --global-batch rows split over the GPUs; "
                         "both (the default for N > 1): weak is the line's value, strong its 'strong' object")
    ap.add_argument("--batch", type=int, default=None,
                    help="samples per GPU (weak scaling; default 2^20, c1 4096)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="samples in all (strong scaling; default 2^20, c1 4096)")
    ap.add_argument("--backend", default=None, choices=("nccl", "gloo"),
                    help="torch.distributed backend for N > 1 (default: nccl = RCCL)")
    ap.add_argument("--parity-rows", type=int, default=None,
                    help="rows checked against the CPU oracle after the timed loop (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timer", action="store_true", help="skip the per-kernel event timer")
    ap.add_argument("--no-status-checks", action="store_true",
                    help="diagnostic builds only (ablations whose results are not valid): no status checks")
    ap.add_argument("--unfused", action="store_true", help="disable the fused MFMA layer kernel")
    ap.add_argument("--no-chain", action="store_true",
                    help="one fused launch per layer instead of one chained launch per run of layers")
    ap.add_argument("--sync-checks", action="store_true",
                    help="status checks with a host sync per call (config.STRICT_CHECKS = True)")
    ap.add_argument("--graph", default="auto", choices=("auto", "on", "off"),
                    help="replay log_prob as one HIP graph (graphs.GraphedLogProb); auto: for the "
                         "small-batch workloads (c1), where launches bound the step")
    ap.add_argument("--dist", action="store_true",
                    help="a process group and the NLL all-reduce even at N = 1 (RCCL on a one-GPU box)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    dflt = DEFAULT_BATCH.get(args.workload, 1 << 20)
    args.batch = dflt if args.batch is None else args.batch
    args.global_batch = dflt if args.global_batch is None else args.global_batch

    from normalizingflow_amd import config, dist as nfdist, kernels
    from normalizingflow_amd import flush_status_checks
    import torch.distributed as dist

    rank, world, local = nfdist.init_from_env(backend=args.backend, force=args.dist)
    use_dist = world > 1 or args.dist
    if world != args.gpus and rank == 0:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    # gloo runs share one device when there are fewer devices than ranks (tests)
    ndev = torch.cuda.device_count()
    device = torch.device("cuda", local if local < ndev else local % max(ndev, 1))
    torch.cuda.set_device(device)
    config.USE_FUSED = not args.unfused
    config.USE_CHAIN = not args.no_chain
    config.STRICT_CHECKS = True if args.sync_checks else "deferred"
    if args.no_status_checks:
        config.STRICT_CHECKS = False
    # N > 1 times both modes by default: weak (the line's value, c4) and strong
    # (the metric's 1M x 64 split over the ranks, in the line's "strong" object)
    scaling = args.scaling or ("both" if world > 1 else "weak")
    modes = ["weak", "strong"] if scaling == "both" else [scaling]

    model, sd, _ = build_model(args.workload, device)
    def graph_for(B):
        """auto: a HIP graph replay where launches are a visible part of the
        step -- the small-batch workloads (c1; the applications' 40-50-row
        NSF_AR and RealNVP-2048 batches) and per-rank batches of at most 2^17
        rows (the 8-GPU strong-scaling shard), where the host-side launch and
        status-copy overhead is ~2 % of a step.  Not poly2048: the replay's
        staleness check over its 12,288 parameters costs more than its two
        launches (1.10 vs 1.04 ms per step, profiles/r6/r6v_*).  A replay
        launches nothing from the host, so the kernel timer (the roofline's
        per-launch means) then times an untimed eager pass of the same K steps
        first."""
        if args.graph != "auto":
            return args.graph == "on"
        # c3 at the metric's 2^20 rows too: its one launch per step replays
        # 0.2-0.5 % faster than the eager call (profiles/r6/r6ai_c3_graph_ab.txt)
        return args.workload in ("c1", "c3") or (B <= (1 << 17) and args.workload != "poly2048")

    def run(mode):
        """One mode's timed loop: W warm-up steps, then K steps bracketed by a
        barrier + synchronize, max over ranks."""
        if mode == "strong":
            lo, hi = nfdist.shard_range(args.global_batch, rank, world)
            B, total = hi - lo, args.global_batch
        else:
            B, total = args.batch, world * args.batch
        use_graph = graph_for(B)
        g = torch.Generator(device=device).manual_seed(rank)
        x = make_x(args.workload, B, g, device)  # resident in HBM before timing
        graphed = None
        if use_graph:
            from normalizingflow_amd.graphs import GraphedLogProb
            graphed = GraphedLogProb(model, x)
        res = {"nll": None}

        def step():
            lp = graphed() if graphed is not None else model.log_prob(x)
            if use_dist:
                res["nll"] = nfdist.nll_allreduce(lp)
            return lp

        progress("%s: %d rows per rank, warm-up" % (mode, B))
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        flush_status_checks()
        progress("%s: timed loop" % mode)
        timer = None
        if not args.no_timer:
            timer = kernels.TIMER = kernels.KernelTimer()
            if graphed is not None:
                # a replay launches nothing from the host to time: the per-kernel
                # means come from an eager pass of the same K steps, outside the
                # timed region
                for _ in range(args.steps):
                    model.log_prob(x)
                torch.cuda.synchronize()
                kernels.TIMER = None
                flush_status_checks()
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            lp = step()
        torch.cuda.synchronize()
        if use_dist:
            dist.barrier()
        dt = time.perf_counter() - t0
        kernels.TIMER = None
        flush_status_checks()  # the reference's errors, if any step raised one
        if use_dist:
            t = torch.tensor([dt], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        progress("%s: %.4f ms per step" % (mode, dt / args.steps * 1e3))
        res.update(mode=mode, B=B, total=total, x=x, lp=lp, dt=dt, graphed=graphed is not None,
                   summary=timer.summary() if timer is not None else {})
        return res

    results = [run(m) for m in modes]
    if rank == 0:
        sd_cpu = {k: v.cpu() for k, v in sd.items()}
        n_par = args.parity_rows if args.parity_rows is not None else \
            (4096 if args.workload == "c5" else 16384)

        def record(r):
            value = r["total"] * args.steps / r["dt"]
            summary = r["summary"]
            dom = max(summary.items(), key=lambda kv: kv[1][2])[0] if summary else None
            rl = roofline(args.workload, summary, r["B"],
                          load_traffic(dom, args.workload, r["B"]) if dom else None, args.steps)
            par = None
            if n_par > 0:
                n = min(n_par, r["B"])
                progress("parity: %d rows vs the CPU oracle" % n)
                par = parity(args.workload, sd_cpu, r["x"][:n].cpu(), r["lp"][:n].cpu())
            return value, rl, par

        main_r = results[0]
        value, rl, par = record(main_r)
        cpu = None
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline is an N=1 figure
            cpu = cpu_baseline(args.workload, sd_cpu)
        desc = WORKLOADS[args.workload][0]
        out = {
            "metric": METRICS[args.workload],
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(main_r["dt"] / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": main_r["mode"],
            "vs_baseline": (round(value / BASELINE_CPU[args.workload], 3)
                            if args.workload in BASELINE_CPU else None),
            "dtype": DTYPE_FUSED if config.USE_FUSED else "fp32",
            "data": ("synthetic two moons (noise 0.05)" if args.workload == "c1" else "synthetic x ~ N(0, I)")
                    + " resident in HBM; random-init weights (seed 1234)",
            "config": {"workload": args.workload + ": " + desc, "global_batch": main_r["total"],
                       "per_gpu_batch": main_r["B"], "parallelism": "dp%d (sample sharding)" % world,
                       "scaling": main_r["mode"],
                       "backend": (args.backend or "nccl") if use_dist else None,
                       "fused_layer_kernel": bool(config.USE_FUSED),
                       "hip_graph": main_r["graphed"],
                       "chained_layers": bool(config.USE_FUSED and config.USE_CHAIN),
                       "status_checks": "sync per call" if args.sync_checks else
                       "deferred (no host sync per step; flushed after the timed loop)",
                       "conditioner_arith": ARITH.get(args.workload) if config.USE_FUSED
                       else "f32 (rocBLAS)"},
            "roofline": rl,
            "parity": par,
            "cpu_baseline": cpu,
            "nll": None if main_r["nll"] is None else float(main_r["nll"]),
            "kernels": {k: {"launches": v[0], "mean_ms": round(v[1], 4)}
                        for k, v in main_r["summary"].items()},
        }
        if len(results) > 1:
            r = results[1]
            v2, rl2, par2 = record(r)
            out["strong"] = {
                "value": round(v2, 1), "unit": "samples/s", "ms_per_step": round(r["dt"] / args.steps * 1e3, 4),
                "global_batch": r["total"], "per_gpu_batch": r["B"], "scaling": "strong",
                "nll": None if r["nll"] is None else float(r["nll"]),
                "roofline": rl2, "parity": par2,
                "note": "the metric's 1M x 64 batch split over the ranks (dist.shard_range), timed in the "
                        "same invocation after the weak loop"}
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
