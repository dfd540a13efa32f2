"""Training path on the GPU: gradients through the kernel-backed layers
(HIP forward + recompute-backward, flows._LayerFn) against the oracle's
autograd on the CPU, for every layer type and both directions; the
reference's training step (applications/src/train.py:22-28: loss =
-mean(prior_lp + log_det), Adam) run side by side for a few steps, which also
checks that the fused kernels re-pack their weights after every optimizer
step; the reverse-KL path (setup.py:90-94) through model.inverse; and
DistributedDataParallel over two ranks (gloo on the box's one device) whose
averaged gradients must equal the full-batch oracle gradient.

Tolerance: gradients agree to max|ours - oracle| <= 1e-4 * max|oracle| per
tensor (both are fp32; the GPU's summation order differs from the CPU's).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn.functional as F

import nf.flows as nff
import nf.flows_1 as nff1
import nf.models as nfm
from oracle import nf_oracle as orc

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
GRAD_TOL = 1e-4


def rel_close(a, b, tol=GRAD_TOL, what="", floor=1e-12):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    scale = max(float(b.abs().max()), floor)
    err = float((a - b).abs().max()) / scale
    assert err <= tol, "%s: rel err %.3g" % (what, err)


def spec_of(layer, prefix):
    if isinstance(layer, nff.NSF_CL):
        return dict(type="NSF_CL", prefix=prefix, size=layer.size, dim=layer.dim, K=layer.K,
                    B=layer.B, mask=[int(m) for m in layer.mask])
    if isinstance(layer, nff.RealNVP):
        return dict(type="RealNVP", prefix=prefix, dim=layer.dim)
    if isinstance(layer, nff1.NSF_AR):
        return dict(type="NSF_AR_flows1", prefix=prefix, dim=layer.dim, K=layer.K, B=layer.B,
                    periodic=layer.periodic)
    if isinstance(layer, nff.NSF_AR):
        return dict(type="NSF_AR", prefix=prefix, dim=layer.dim, K=layer.K, B=layer.B)
    if isinstance(layer, nff.Planar):
        return dict(type="Planar", prefix=prefix, nonlinearity=layer.h.__name__)
    if isinstance(layer, nff.Radial):
        return dict(type="Radial", prefix=prefix)
    if isinstance(layer, nff.MAF):
        return dict(type="MAF", prefix=prefix, dim=layer.dim)
    if isinstance(layer, nff.ActNorm):
        return dict(type="ActNorm", prefix=prefix)
    if isinstance(layer, nff.OneByOneConv):
        return dict(type="OneByOneConv", prefix=prefix)
    raise TypeError(type(layer))


def _actnorm(d):
    a = nff.ActNorm(d)
    with torch.no_grad():
        a.mu.normal_(0, 0.5)
        a.log_sigma.normal_(0, 0.3)
    return a


def _radial(d):
    r = nff.Radial(d)
    r.reset_parameters(d)
    return r


LAYERS = {
    # c3's layer: the fused MFMA NSF kernel
    "nsfcl_fused": (lambda: nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[0]), 64, True),
    # 3 coordinates, non-prefix mask: FCNN + nfk_rqs_coupling
    "nsfcl_unfused": (lambda: nff.NSF_CL(size=6, dim=3, K=5, B=3, hidden_dim=24, mask=[1]), 18, True),
    "realnvp_fused": (lambda: nff.RealNVP(64, hidden_dim=100), 64, True),
    # half-dimension 5 runs zero-padded to 16 on the fused kernel (RealNVP._fused_half)
    "realnvp_padded": (lambda: nff.RealNVP(10, hidden_dim=20), 10, True),
    # H = 140 is past the fused kernels: library GEMM conditioners + nfk_affine_coupling
    "realnvp_unfused": (lambda: nff.RealNVP(10, hidden_dim=140), 10, True),
    "nsfar": (lambda: nff.NSF_AR(dim=4, K=5, B=3, hidden_dim=16), 4, True),
    "nsfar1": (lambda: nff1.NSF_AR(dim=4, K=5, B=3, hidden_dim=16), 4, True),
    "nsfar1_plain": (lambda: nff1.NSF_AR(dim=3, K=4, B=3, hidden_dim=12, periodic=False), 3, True),
    "planar_tanh": (lambda: nff.Planar(6), 6, False),
    "planar_elu": (lambda: nff.Planar(6, nonlinearity=F.elu), 6, False),
    "planar_leaky": (lambda: nff.Planar(6, nonlinearity=F.leaky_relu), 6, False),
    "radial": (lambda: _radial(6), 6, False),
    "maf": (lambda: nff.MAF(6, hidden_dim=8), 6, True),
    "actnorm": (lambda: _actnorm(6), 6, True),
    "onebyone": (lambda: nff.OneByOneConv(6), 6, True),
}


def _layer_case(name, inverse):
    make, d, has_inv = LAYERS[name]
    if inverse and not has_inv:
        pytest.skip("no inverse")
    torch.manual_seed(11)
    layer = make()
    x = torch.randn(1024, d, generator=torch.Generator().manual_seed(3)) * 1.5
    g = torch.Generator().manual_seed(4)
    gz = torch.randn(1024, d, generator=g)
    gld = torch.randn({"radial": (1,), "actnorm": (), "onebyone": ()}.get(name, (1024,)), generator=g)
    return layer, x, gz, gld


@pytest.mark.parametrize("inverse", [False, True])
@pytest.mark.parametrize("name", list(LAYERS))
def test_layer_grads_vs_oracle(name, inverse, hip_device):
    layer, x, gz, gld = _layer_case(name, inverse)
    # oracle: autograd of the CPU restatement
    sd = {"l." + k: v.detach().clone().requires_grad_(True) for k, v in layer.named_parameters()}
    if isinstance(layer, nff.OneByOneConv):
        sd["l.P"] = layer.P.clone()
    xr = x.clone().requires_grad_(True)
    zr, ldr = orc.apply_layer(spec_of(layer, "l."), xr, sd, inverse=inverse)
    ((zr * gz).sum() + (ldr * gld).sum()).backward()
    # ours
    layer = layer.to(hip_device)
    xg = x.to(hip_device).requires_grad_(True)
    z, ld = layer.inverse(xg) if inverse else layer(xg)
    assert z.requires_grad and ld.requires_grad
    ((z * gz.to(hip_device)).sum() + (ld * gld.to(hip_device)).sum()).backward()
    rel_close(z, zr, 1e-5, "z")
    # log|det| of an orthogonal 1x1 conv is ~1e-7: compare on an O(1) scale
    rel_close(ld.expand_as(ldr), ldr, 1e-5, "logdet", floor=1.0)
    rel_close(xg.grad, xr.grad, what="x.grad")
    for k, p in layer.named_parameters():
        ref = sd["l." + k].grad
        if ref is None:
            assert p.grad is None or not bool(p.grad.any()), k
        else:
            rel_close(p.grad, ref, what=k)


# the hand-written backward of each layer class and the kernels it must launch
NATIVE_BWD = {
    "planar_tanh": {"nfk_planar_bwd"},
    "planar_leaky": {"nfk_planar_bwd"},
    "radial": {"nfk_radial_bwd_scalars", "nfk_radial_bwd_apply"},
    "actnorm": {"nfk_actnorm_bwd"},
    "maf": {"nfk_maf_bwd"},
    "nsfar": {"nfk_rqs_coupling_bwd", "nfk_trig_features_bwd"},
    "nsfar1": {"nfk_rqs_coupling_bwd", "nfk_trig_features_bwd"},
    "nsfar1_plain": {"nfk_rqs_coupling_bwd"},
    "realnvp_unfused": {"nfk_affine_coupling_bwd"},
    "realnvp_padded": {"nfk_affine_coupling_bwd"},
    "nsfcl_fused": {"nfk_fused_nsf_vjp"},
    "onebyone": set(),  # library GEMMs (no kernel of ours), but not the recompute
}


@pytest.mark.parametrize("inverse", [False, True])
@pytest.mark.parametrize("name", list(NATIVE_BWD))
def test_backward_runs_native_kernels(name, inverse, hip_device):
    """Each layer's backward is its hand-written VJP on the HIP kernels, not
    the autograd recompute of torch_math (nothing of it may be called)."""
    from normalizingflow_amd import kernels as K_, torch_math
    layer, x, gz, gld = _layer_case(name, inverse)
    layer = layer.to(hip_device)
    xg = x.to(hip_device).requires_grad_(True)
    z, ld = layer.inverse(xg) if inverse else layer(xg)
    loss = (z * gz.to(hip_device)).sum() + (ld * gld.to(hip_device)).sum()
    prev, prev_fwd = K_.TIMER, torch_math.layer_forward
    K_.TIMER = K_.KernelTimer()

    def _no_recompute(*a, **k):
        raise AssertionError("autograd recompute used for %s" % name)
    torch_math.layer_forward = _no_recompute
    try:
        loss.backward()
        torch.cuda.synchronize()
        launched = set(K_.TIMER.summary())
    finally:
        K_.TIMER, torch_math.layer_forward = prev, prev_fwd
    assert NATIVE_BWD[name] <= launched, launched
    assert xg.grad is not None and all(p.grad is not None for p in layer.parameters())


@pytest.mark.parametrize("name", ["planar_tanh", "radial", "actnorm"])
def test_backward_batch_reductions_large(name, hip_device):
    """Parameter gradients are batch sums over many row chunks (70,000 rows:
    the column reductions' chunk cap): oracle autograd in fp64 as reference."""
    make, d, _ = LAYERS[name]
    torch.manual_seed(5)
    layer = make()
    B = 70000
    x = torch.randn(B, d, generator=torch.Generator().manual_seed(6))
    g = torch.Generator().manual_seed(7)
    gz = torch.randn(B, d, generator=g)
    gld = torch.randn({"radial": (1,), "actnorm": ()}.get(name, (B,)), generator=g)
    sd = {"l." + k: v.detach().double().clone().requires_grad_(True) for k, v in layer.named_parameters()}
    xr = x.double().requires_grad_(True)
    zr, ldr = orc.apply_layer(spec_of(layer, "l."), xr, sd, inverse=False)
    ((zr * gz.double()).sum() + (ldr * gld.double()).sum()).backward()
    layer = layer.to(hip_device)
    xg = x.to(hip_device).requires_grad_(True)
    z, ld = layer(xg)
    ((z * gz.to(hip_device)).sum() + (ld * gld.to(hip_device)).sum()).backward()
    rel_close(xg.grad, xr.grad, what="x.grad")
    for k, p in layer.named_parameters():
        rel_close(p.grad, sd["l." + k].grad, what=k)


def _c3(n_layers, seed=1234, hidden=100):
    torch.manual_seed(seed)
    flows = [nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=hidden, mask=[i % 2])
             for i in range(n_layers)]
    prior = torch.distributions.MultivariateNormal(torch.zeros(64), torch.eye(64))
    return nfm.NormalizingFlowModel(prior, flows)


def _to_dev(model, dev):
    model.prior = torch.distributions.MultivariateNormal(torch.zeros(64, device=dev),
                                                        torch.eye(64, device=dev))
    return model.to(dev)


def _specs(model):
    return [spec_of(f, "flows.%d." % i) for i, f in enumerate(model.flows)]


def test_train_steps_match_oracle(hip_device):
    """train.py:22-28 for 3 optimizer steps on the GPU model and on the oracle
    with the same initial weights and batches: per-step loss and gradients,
    and the final weights.  SGD with momentum (its update is proportional to
    the gradient, so the final weights inherit the gradient tolerance; Adam's
    sign-like update of ~0 gradients would amplify fp32 summation noise)."""
    model = _c3(2)
    specs = _specs(model)
    ref = {k: v.detach().clone().requires_grad_(True) for k, v in model.named_parameters()}
    opt_ref = torch.optim.SGD(list(ref.values()), lr=0.05, momentum=0.9)
    model = _to_dev(model, hip_device)
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
    g = torch.Generator().manual_seed(9)
    for step in range(3):
        x = torch.randn(2048, 64, generator=g)
        opt_ref.zero_grad()
        _, plp, ld = orc.model_forward(specs, ref, x)
        loss_ref = -torch.mean(plp + ld)
        loss_ref.backward()
        opt.zero_grad()
        z, plp_g, ld_g = model(x.to(hip_device))
        loss = -torch.mean(plp_g + ld_g)
        loss.backward()
        assert abs(float(loss.detach()) - float(loss_ref.detach())) <= 1e-5 * abs(float(loss_ref.detach())), step
        for k, p in model.named_parameters():
            rel_close(p.grad, ref[k].grad, what="step%d %s" % (step, k))
        opt_ref.step()
        opt.step()
    for k, p in model.named_parameters():
        rel_close(p, ref[k], 1e-5, "final " + k)
    # inference after training uses the re-packed weights
    with torch.no_grad():
        x = torch.randn(512, 64, generator=g)
        lp_ref = orc.model_log_prob(specs, {k: v.detach() for k, v in ref.items()}, x)
        rel_close(model.log_prob(x.to(hip_device)), lp_ref, 1e-5, "log_prob after training")


def test_reverse_kl_grads(hip_device):
    """setup.py:90-94 reverseKL through model.inverse (gradient w.r.t. the
    prior draws and the weights)."""
    model = _c3(2, seed=7)
    specs = _specs(model)
    ref = {k: v.detach().clone().requires_grad_(True) for k, v in model.named_parameters()}
    z = torch.randn(1024, 64, generator=torch.Generator().manual_seed(2))
    zr = z.clone().requires_grad_(True)
    xr, ldr = orc.model_inverse(specs, ref, zr)
    loss_ref = torch.mean(xr.pow(2).sum(1)) + torch.mean(orc.normal_log_prob(zr) - ldr)
    loss_ref.backward()
    model = _to_dev(model, hip_device)
    zg = z.to(hip_device).requires_grad_(True)
    x, ld = model.inverse(zg)
    loss = torch.mean(x.pow(2).sum(1)) + torch.mean(model.prior.log_prob(zg) - ld)
    loss.backward()
    rel_close(loss, loss_ref, 1e-5, "loss")
    rel_close(zg.grad, zr.grad, what="z.grad")
    for k, p in model.named_parameters():
        rel_close(p.grad, ref[k].grad, what=k)


def test_no_grad_path_unchanged(hip_device):
    """With grad enabled but nothing requiring grad, the in-place chain runs
    (no autograd nodes) and evaluate() never builds a graph."""
    model = _to_dev(_c3(2), hip_device)
    x = torch.randn(256, 64, device=hip_device)
    for p in model.parameters():
        p.requires_grad_(False)
    z, plp, ld = model(x)
    assert not z.requires_grad
    for p in model.parameters():
        p.requires_grad_(True)
    lp = model.evaluate(x)
    assert not lp.requires_grad
    z2, plp2, ld2 = model(x)
    assert z2.requires_grad
    rel_close(z2, z, 1e-6, "z")
    rel_close(plp2 + ld2, lp, 1e-5, "log_prob")


# --------------------------------------------------------------------------- DDP
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _build_mixed(seed):
    torch.manual_seed(seed)
    flows = [_radial(64)] + [nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[i % 2])
                             for i in range(2)]
    prior = torch.distributions.MultivariateNormal(torch.zeros(64), torch.eye(64))
    return nfm.NormalizingFlowModel(prior, flows)


def _ddp_worker(rank, world, port, x, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    try:
        import torch.distributed as dist
        from normalizingflow_amd import dist as nfd
        nfd.init_from_env(backend="gloo")
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        model = _to_dev(_build_mixed(21), dev)
        ddp = nfd.data_parallel(model, device=dev)
        xs = nfd.shard(x).to(dev)
        z, plp, ld = ddp(xs)
        loss = nfd.sharded_nll(plp + ld)  # exact for the uneven shards of x
        loss.backward()
        # numpy: pickled by value (a torch CPU tensor would be shared through a
        # file descriptor that vanishes when this process exits)
        q.put((rank, {k: p.grad.cpu().numpy() for k, p in model.named_parameters()}))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        q.put((rank, traceback.format_exc() + repr(e)))


@pytest.mark.parametrize("world,rows", [(2, 4096), (3, 4097)])
def test_ddp_grads_equal_full_batch(world, rows):
    """DDP over ``world`` ranks (3 ranks: 4097 rows, shards 1366/1366/1365)
    with dist.sharded_nll: every rank's averaged gradient is the full-batch
    oracle gradient of -mean(log p)."""
    model = _build_mixed(21)
    specs = [spec_of(f, "flows.%d." % i) for i, f in enumerate(model.flows)]
    ref = {k: v.detach().clone().requires_grad_(True) for k, v in model.named_parameters()}
    x = torch.randn(rows, 64, generator=torch.Generator().manual_seed(8)) * 0.8
    _, plp, ld = orc.model_forward(specs, ref, x)
    (-torch.mean(plp + ld)).backward()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ddp_worker, args=(r, world, port, x, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    for rank, grads in out:
        assert isinstance(grads, dict), grads
        for k, g in grads.items():
            rel_close(torch.from_numpy(g), ref[k].grad, what="rank%d %s" % (rank, k))


# --------------------------------------------------------------------------- kernel
def _spline_ref(mode, x, u, K, B, inverse):
    """Reference function of the raw per-element parameters for each param_mode."""
    uw, uh, ud = u[..., :K], u[..., K:2 * K], u[..., 2 * K:]
    if mode == 0:   # NSF_CL raw conditioner output (flows.py:233-236)
        return orc.unconstrained_rq_spline(x, 2 * B * torch.softmax(uw, -1),
                                           2 * B * torch.softmax(uh, -1), F.softplus(ud),
                                           inverse=inverse, tail_bound=B, strict=False)
    if mode == 1:   # unconstrained_RQS arguments (utils.py:27)
        return orc.unconstrained_rq_spline(x, uw, uh, ud, inverse=inverse, tail_bound=B,
                                           strict=False)
    y, lad, _ = orc.rq_spline(x, uw, uh, ud, inverse=inverse, left=-B, right=B, bottom=-B, top=B)
    return y, lad


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("K", [3, 8, 16])
@pytest.mark.parametrize("inverse", [False, True])
def test_rqs_coupling_bwd_kernel_vs_fp64_autograd(mode, K, inverse, hip_device):
    """nfk_rqs_coupling_bwd against the fp64 autograd of the oracle spline, with
    inputs inside and outside [-B, B] (identity tails) and gz, gld both live."""
    from normalizingflow_amd import kernels as K_
    n, n_up, B = 2048, 4, 3.0
    P = 3 * K + 1 if mode == 2 else 3 * K - 1
    g = torch.Generator().manual_seed(K * 7 + mode)
    scale = 3.5 if mode != 2 else 2.9   # mode 2 has no tails: stay inside
    x = (torch.rand(n, n_up, generator=g) * 2 - 1) * scale
    u = torch.randn(n, n_up, P, generator=g)
    gz = torch.randn(n, n_up, generator=g)
    gld = torch.randn(n, generator=g)
    x64, u64 = x.double().requires_grad_(True), u.double().requires_grad_(True)
    y, lad = _spline_ref(mode, x64, u64, K, B, inverse)
    ((y * gz.double()).sum() + (lad.sum(1) * gld.double()).sum()).backward()
    dev = hip_device
    idx = torch.arange(n_up, dtype=torch.int32, device=dev)
    gp = torch.empty(n, n_up * P, device=dev)
    gx = torch.empty(n, n_up, device=dev)
    K_.rqs_coupling_bwd(x.to(dev), u.reshape(n, -1).contiguous().to(dev), idx, idx, gz.to(dev),
                        gld.to(dev), gp, gx, K=K, left=-B, right=B, bottom=-B, top=B,
                        tails=(mode != 2), param_mode=mode, inverse=inverse)
    torch.cuda.synchronize()
    # the fp32 autograd of the same function (what the reference computes)
    # sets the bar: ours must be within 2e-4 of fp64 or on par with it
    x32, u32 = x.clone().requires_grad_(True), u.clone().requires_grad_(True)
    y32, lad32 = _spline_ref(mode, x32, u32, K, B, inverse)
    ((y32 * gz).sum() + (lad32.sum(1) * gld).sum()).backward()
    for name, ours, r32, r64 in (("gx", gx, x32.grad, x64.grad),
                                 ("gparams", gp.reshape(n, n_up, P), u32.grad, u64.grad)):
        scale = float(r64.abs().max())
        e32 = float((r32.double() - r64).abs().max()) / scale
        rel_close(ours, r64, max(2e-4, 4 * e32), name)
    out = ~((x >= -B) & (x <= B))
    if mode != 2 and bool(out.any()):
        assert torch.equal(gx.cpu()[out], gz[out])
        assert bool((gp.cpu().reshape(n, n_up, P)[out] == 0).all())


def test_app_train_steps_reduce_nll(hip_device, tmp_path):
    """normalizingflow_amd.app: a config-built NSF_CL model (setup.py:55-63) trained
    by train_step (train.py:21-29) on the device lowers the NLL of a shifted
    Gaussian, and its checkpoint reloads to the same log_prob."""
    from normalizingflow_amd import app
    cfg = app.get_cfg_defaults()
    cfg.device = "cuda:0"
    cfg.dataset.nparticles, cfg.dataset.dim = 8, 3
    cfg.dataset.ncellx, cfg.dataset.cell_len = 2, 3.0
    cfg.prior.type, cfg.prior.nparticles, cfg.prior.dim = "Normal", 8, 3
    cfg.flow.type, cfg.flow.nlayers, cfg.flow.nsplines, cfg.flow.hidden_dim = "NSF_CL", 3, 8, 32
    torch.manual_seed(0)
    model = app.build_model(cfg)
    opt = torch.optim.Adam(model.parameters(), lr=3e-3)
    g = torch.Generator(device=hip_device).manual_seed(1)
    xs = [torch.randn(4096, 24, device=hip_device, generator=g) * 0.7 + 0.4 for _ in range(40)]
    losses = [float(app.train_step(model, opt, x)) for x in xs]
    assert losses[-1] < losses[0] - 0.5, losses[::8]
    path = str(tmp_path / "ck.pth")
    app.save_checkpoint(path, model, opt, epoch=40, losses=losses)
    torch.manual_seed(5)
    other = app.build_model(cfg)
    app.load_checkpoint(other, path)
    with torch.no_grad():
        rel_close(other.log_prob(xs[0]), model.log_prob(xs[0]), 0.0, "reloaded log_prob")


@pytest.mark.parametrize("name", ["planar_tanh", "radial", "actnorm", "maf"])
def test_backward_bitwise_reproducible(name, hip_device):
    """The parameter gradients are batch sums formed in a fixed order (no
    atomics, nfk_flows_bwd.hip): two backward passes agree bit for bit."""
    make, d, _ = LAYERS[name]
    torch.manual_seed(21)
    layer = make().to(hip_device)
    x = torch.randn(5000, d, device=hip_device)
    gz = torch.randn(5000, d, device=hip_device)
    got = []
    for _ in range(2):
        layer.zero_grad(set_to_none=True)
        xg = x.clone().requires_grad_(True)
        z, ld = layer(xg)
        ((z * gz).sum() + ld.sum()).backward()
        got.append([xg.grad.clone()] + [p.grad.clone() for p in layer.parameters()])
    for a, b in zip(*got):
        assert torch.equal(a, b)
