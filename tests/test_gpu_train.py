"""GPU parity of the fused training step through the C ABI.

  nlosgr_mse   vs the fp64 expression of compute_loss (nlos_helpers.py:323-327):
               loss / equal_loss rel <= 1e-5, grad vs the torch fp32 expression rel <= 1e-6
  nlosgr_adam  vs torch.optim.Adam(eps=1e-15) with the reference's six groups
               (gaussian_model.py:223-242) over 5 steps: params / moments rel <= 1e-6 of max
  TrainStep    vs the same iteration composed from torch pieces (RenderFn autograd + torch MSE
               [+ the optional regularisers] + torch.optim.Adam, main.py:198-214) on identical
               inputs over 3 iterations: params rel <= 1e-5 of max
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("n", [1, 1000, 257 * 1031, 3 * 1024 * 1024 + 5])
def test_mse_matches_torch(n):
    from nlosgr.train import mse
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(n)
    hist = torch.rand(n, generator=g).to(dev)
    target = (torch.rand(n, generator=g) * 1e-2).to(dev)
    gt_times = 100.0
    loss2, grad = mse(hist, target, gt_times, grad_scale=0.5)
    t = target.double() * gt_times
    d = hist.double() - t
    ref_loss = (d * d).mean()
    ref_eq = ref_loss / (t * t).mean()
    assert abs(loss2[0].item() - ref_loss.item()) <= 1e-5 * ref_loss.item()
    assert abs(loss2[1].item() - ref_eq.item()) <= 1e-5 * ref_eq.item()
    # gradient of 0.5 * mean((hist - gt target)^2) w.r.t. hist
    ref_grad = (0.5 * 2.0 / n) * (hist - target * gt_times)
    assert _rel(grad, ref_grad) <= 1e-6


def test_mse_empty_and_errors():
    from nlosgr import _lib
    from nlosgr.train import mse
    dev = torch.device("cuda:0")
    e = torch.empty(0, device=dev)
    loss2, grad = mse(e, e)
    assert loss2.tolist() == [0.0, 0.0] and grad.numel() == 0
    with pytest.raises(ValueError):
        mse(torch.zeros(4, device=dev), torch.zeros(5, device=dev))
    lib = _lib.load()
    assert lib.nlosgr_mse(None, None, 1.0, -1, 1.0, None, None, None, None) != 0
    assert b"n must be" in lib.nlosgr_last_error()


def _groups(dev, ng=5000, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    shapes = [(ng, 3), (ng, 1), (ng, 15), (ng,), (ng, 3), (ng, 4)]
    return [torch.randn(*s, generator=g).to(dev) for s in shapes]


def test_adam_matches_torch_optim():
    from nlosgr.train import Adam
    dev = torch.device("cuda:0")
    ours = [t.clone() for t in _groups(dev)]
    ref = [torch.nn.Parameter(t.clone()) for t in ours]
    lrs = [1.6e-4, 2.5e-3, 2.5e-3 / 20, 2.5e-2, 5e-3, 1e-3]
    opt = torch.optim.Adam([{"params": [p], "lr": lr} for p, lr in zip(ref, lrs)], lr=0.0, eps=1e-15,
                           foreach=False)
    mine = Adam(ours, eps=1e-15)
    g = torch.Generator(device="cpu").manual_seed(7)
    for step in range(5):
        grads = [(torch.randn(p.shape, generator=g) * 10.0 ** (step - 3)).to(dev) for p in ours]
        step_lrs = [lr * (0.9 ** step) for lr in lrs]
        for p, gr, lr, grp in zip(ref, grads, step_lrs, opt.param_groups):
            p.grad = gr.clone()
            grp["lr"] = lr
        opt.step()
        mine.step(grads, step_lrs)
    torch.cuda.synchronize()
    for a, b in zip(ours, ref):
        assert _rel(a, b) <= 1e-6
    for i, b in enumerate(ref):
        st = opt.state[b]
        assert _rel(mine.exp_avg[i], st["exp_avg"]) <= 1e-6
        assert _rel(mine.exp_avg_sq[i], st["exp_avg_sq"]) <= 1e-6


def test_adam_rejects_bad_args():
    from nlosgr import _lib
    from nlosgr.train import Adam
    dev = torch.device("cuda:0")
    with pytest.raises(ValueError):
        Adam([torch.zeros(3, device=dev, dtype=torch.float64)])
    with pytest.raises(ValueError):
        Adam([torch.zeros(3, device=dev)] * 9)
    lib = _lib.load()
    arr = (_lib.AdamGroup * 1)()
    assert lib.nlosgr_adam(arr, 1, 0, 0.9, 0.999, 1e-15, None) != 0
    assert b"step" in lib.nlosgr_last_error()


def _scene_model(dev, ng=400, H=6, W=5, T=48, seed=3, cutoff=3.0):
    from nlosgr import GaussianParams
    from nlosgr.volume import Scene, make_config
    scene = Scene(H=H, W=W, T=T, ns=8)
    model = GaussianParams.synthetic(ng, 3, preset="cuda", device=dev, seed=seed)
    geo = scene.geometry(dev, "cuda", "noocl")
    cfg = make_config(model, scene, "cuda", "noocl", cutoff=cutoff)
    g = torch.Generator().manual_seed(seed + 1)
    target = (torch.rand(H * W, T, generator=g) * 1e-3).to(dev)
    return scene, model, geo, cfg, target


@pytest.mark.parametrize("regularization", [False, True])
def test_train_step_matches_torch_composition(regularization):
    """Three fused TrainStep iterations == render autograd + torch MSE + torch.optim.Adam."""
    from nlosgr import GaussianParams
    from nlosgr.train import OptimizationParams, TrainStep
    from nlosgr.volume import render_volume
    dev = torch.device("cuda:0")
    scene, model, geo, cfg, target = _scene_model(dev)
    twin = GaussianParams(*(p.detach().clone() for p in model.parameters()), model.active_sh_degree)
    gt_times = 100.0
    opt = OptimizationParams(regularization=regularization)
    step = TrainStep(model, geo, cfg, target, gt_times=gt_times, opt=opt, spatial_lr_scale=2.0)
    names = ["mu", "scaling", "rotation", "opacity", "f_dc", "f_rest"]     # GaussianParams.parameters() order
    by_name = dict(zip(names, twin.parameters()))
    lr0 = {"mu": opt.position_lr_init * 2.0, "f_dc": opt.feature_lr, "f_rest": opt.feature_lr / 20.0,
           "opacity": opt.opacity_lr, "scaling": opt.scaling_lr, "rotation": opt.rotation_lr}
    order = ["mu", "f_dc", "f_rest", "opacity", "scaling", "rotation"]       # gaussian_model.py:229-236
    torch_opt = torch.optim.Adam([{"params": [by_name[n]], "lr": lr0[n], "name": n} for n in order], lr=0.0,
                                 eps=1e-15, foreach=False)
    for it in range(3):
        loss2 = step(it)
        torch_opt.param_groups[0]["lr"] = step.learning_rates(it)[0]
        torch_opt.zero_grad()
        hist = render_volume(twin, geo, cfg)
        t = target * gt_times
        loss = ((hist - t) ** 2).mean()
        if regularization:
            loss = loss + opt.opacity_reg * torch.abs(torch.sigmoid(twin._opacity)).mean()
            loss = loss + opt.scale_reg * torch.abs(torch.exp(twin._scaling)).mean()
        loss.backward()
        torch_opt.step()
        assert abs(loss2[0].item() - loss.item()) <= 1e-5 * loss.item()
    torch.cuda.synchronize()
    for n, a, b in zip(names, model.parameters(), twin.parameters()):
        assert _rel(a, b) <= 1e-5, n


def test_train_step_checkpoint_resume(tmp_path):
    """Two iterations, checkpoint, resume in a fresh TrainStep, one more iteration == three
    uninterrupted iterations (Adam moments, step count and lr schedule restored)."""
    from nlosgr import GaussianParams
    from nlosgr.checkpoint import load_checkpoint, save_checkpoint
    from nlosgr.train import TrainStep
    dev = torch.device("cuda:0")
    scene, model, geo, cfg, target = _scene_model(dev)
    twin = GaussianParams(*(p.detach().clone() for p in model.parameters()), model.active_sh_degree)
    a = TrainStep(model, geo, cfg, target, gt_times=100.0)
    for _ in range(3):
        a()
    b = TrainStep(twin, geo, cfg, target, gt_times=100.0)
    for _ in range(2):
        b()
    f = tmp_path / "ck.pt"
    save_checkpoint(str(f), twin, b)
    fresh = GaussianParams(*(torch.zeros_like(p) for p in twin.parameters()), 0, twin.max_sh_degree)
    c = TrainStep(fresh, geo, cfg, target, gt_times=100.0)
    load_checkpoint(str(f), dev, train_step=c)
    assert c.iteration == 2 and c.adam.step_count == 2
    c()
    torch.cuda.synchronize()
    for p, q in zip(model.parameters(), fresh.parameters()):
        assert _rel(q, p) <= 1e-6


def test_train_step_with_mcmc_density_control():
    """relocate_gs + add_new_gs (nlosgr.densify) between fused steps: dead Gaussians revived, the
    model grows by 5 %, Adam moments follow (zero for new / resampled entries) and training goes on."""
    from nlosgr.densify import add_new_gs, prune_dead_mask, relocate_gs
    from nlosgr.train import TrainStep
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    scene, model, geo, cfg, target = _scene_model(dev)
    step = TrainStep(model, geo, cfg, target, gt_times=100.0)
    step()
    model._opacity.data[:10] = -12.0
    dead = prune_dead_mask(model)
    assert int(dead.sum()) >= 10
    relocate_gs(model, dead, train_step=step)
    assert int(prune_dead_mask(model).sum()) == 0
    ng0 = model._mu.shape[0]
    added = add_new_gs(model, cap_max=10 * ng0, train_step=step)
    assert added == int(1.05 * ng0) - ng0 and model._mu.shape[0] == ng0 + added
    assert step.adam.exp_avg[0].shape[0] == ng0 + added
    assert float(step.adam.exp_avg[0][ng0:].abs().sum()) == 0.0
    loss2 = step()
    torch.cuda.synchronize()
    assert torch.isfinite(loss2).all()
    for p in model.parameters():
        assert torch.isfinite(p).all() and p.shape[0] == ng0 + added


def test_bucketed_backward_equals_full():
    """The backward restricted to Gaussian ranges (nlosgr_options.g_begin/g_end, the buckets of the
    overlapped all-reduce) writes exactly the full backward's rows: bitwise equal."""
    from nlosgr import features_flat
    from nlosgr.render import render_backward, render_forward
    from nlosgr.train import bucket_bounds
    dev = torch.device("cuda:0")
    scene, model, geo, cfg, target = _scene_model(dev, ng=1500)
    args = (model._mu.detach(), model._scaling.detach(), model._rotation.detach(), model._opacity.detach(),
            features_flat(model).detach().contiguous())
    hist, _, ws = render_forward(*args, geo, cfg, ray_cache=True)
    grad = torch.randn_like(hist)
    full = render_backward(*args, geo, cfg, grad_hist=grad, workspace=ws, ray_cache=True)
    outs = tuple(torch.full_like(t, float("nan")) for t in full)
    bounds = bucket_bounds(1500, 4)
    assert bounds == [(0, 512), (512, 1024), (1024, 1500)]
    for gr in bounds:
        render_backward(*args, geo, cfg, grad_hist=grad, workspace=ws, ray_cache=True, g_range=gr, out=outs)
    for a, b in zip(outs, full):
        assert torch.equal(a, b)
    with pytest.raises(RuntimeError):
        render_backward(*args, geo, cfg, grad_hist=grad, g_range=(100, 300))   # not a multiple of 256


def _shard_worker(rank, world, port, out, cutoff=3.0):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nlosgr.distributed import wall_rows
        from nlosgr.train import TrainStep
        dev = torch.device("cuda:0")
        scene, model, geo, cfg, target = _scene_model(dev, ng=1500, cutoff=cutoff)
        idx = wall_rows(scene.H, scene.W, rank, world, device=dev)   # the split bench.py --gpus N uses
        step = TrainStep(model, geo.rows(idx), cfg, target[idx].contiguous(), gt_times=100.0, buckets=4)
        losses = [step(it).cpu() for it in range(2)]
        torch.cuda.synchronize()
        out[rank] = ([p.detach().cpu() for p in model.parameters()], losses)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cutoff", [3.0, 5.7])
def test_sharded_train_step_matches_single_process(cutoff):
    """Two gloo ranks sharing the GPU, each training its row-interleaved wall shard (wall_rows, as
    bench.py --gpus N shards; bucketed, overlapped gradient all-reduce, TrainStep.buckets = 4) ==
    one process training the whole wall.  At 5.7 sigma (no ray cache) both run the slab-
    ordered forward and backward, so the bucketed exchange sums permuted gradient rows and scatters
    them back on every rank."""
    import socket
    import torch.multiprocessing as mp
    from nlosgr.train import TrainStep
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = mp.Manager().dict()
    mp.spawn(_shard_worker, args=(2, port, out, cutoff), nprocs=2, join=True)
    dev = torch.device("cuda:0")
    scene, model, geo, cfg, target = _scene_model(dev, ng=1500, cutoff=cutoff)
    step = TrainStep(model, geo, cfg, target, gt_times=100.0)
    losses = [step(it).cpu() for it in range(2)]
    for r in range(2):
        params, rl = out[r]
        for a, b in zip(rl, losses):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=0)
        for n, a, b in zip(["mu", "scaling", "rotation", "opacity", "f_dc", "f_rest"], params, model.parameters()):
            # band sums add in another order: Adam's first steps ~ lr sign(g) can flip a near-zero gradient
            bad = ((a - b.detach().cpu()).abs() > 1e-5 * (1 + b.detach().cpu().abs())).float().mean().item()
            assert bad < 2e-3, (n, bad)


def test_train_step_orders_match_given_order():
    """at 5.7 sigma (no ray cache) TrainStep renders the forward and the backward on
    slab-permuted Gaussians and scatters the six gradients back; its gradients and loss equal those of
    the step in the given order up to fp32 summation order (2e-5 of each tensor's max; rotation 2e-4)."""
    from nlosgr.train import TrainStep
    dev = torch.device("cuda:0")
    grads, losses = [], []
    for order in ("slab", None):
        scene, model, geo, cfg, target = _scene_model(dev, ng=3000, H=8, W=8, T=64, cutoff=5.7)
        step = TrainStep(model, geo, cfg, target, gt_times=100.0, keep_grads=True, bwd_order=order, fwd_order=order)
        assert (step.fwd_order, step.bwd_order) == (order, order)
        losses.append(step().cpu())
        grads.append([g.detach().cpu() for g in step.grads])
    torch.testing.assert_close(losses[0], losses[1], rtol=2e-6, atol=0)
    for name, a, b in zip(("mu", "f_dc", "f_rest", "opacity", "scaling", "rotation"), *grads):
        err = float((a - b).abs().max() / b.abs().max())
        tol = 2e-4 if name == "rotation" else 2e-5   # (the quaternion Jacobian cancels: test_gpu_fullsize)
        assert float(b.abs().max()) > 0 and err <= tol, (name, err)


def _rccl_worker(rank, world, port, out):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world)   # RCCL on ROCm
    try:
        from nlosgr.train import BucketedAllReduce, allreduce_step, bucket_bounds
        dev = torch.device("cuda:0")
        g = torch.Generator().manual_seed(2)
        ng = 1300
        grads = [torch.randn(ng, 3, generator=g).to(dev), torch.randn(ng, 1, generator=g).to(dev),
                 torch.randn(ng, 15, generator=g).to(dev), torch.randn(ng, generator=g).to(dev),
                 torch.randn(ng, 3, generator=g).to(dev), torch.randn(ng, 4, generator=g).to(dev)]
        ref = [t.clone() for t in grads]
        loss4 = torch.tensor([0.5, 2.0, 10.0, 5.0], device=dev)
        out_g, loss2 = allreduce_step([t.clone() for t in grads], loss4, 20)
        ex = BucketedAllReduce([t.clone() for t in grads], bucket_bounds(ng, 4), None)
        for b in range(len(bucket_bounds(ng, 4))):
            ex.launch(b)
        bucketed = ex.finish()
        torch.cuda.synchronize()
        out[rank] = ([t.cpu() for t in ref], [t.cpu() for t in out_g], [t.cpu() for t in bucketed], loss2.cpu())
    finally:
        dist.destroy_process_group()


def test_rccl_exchange_single_rank():
    """The gradient exchange on the RCCL ("nccl") backend itself, on device buffers: the packed
    all-reduce (allreduce_step) and the bucketed overlapped one (BucketedAllReduce) on a one-rank
    group return the inputs unchanged and the global loss (sum of squared errors / n, se / st).
    One GPU cannot host two RCCL ranks (duplicate device), so the two-rank exchange is covered on
    gloo (test_sharded_train_step_matches_single_process, tests/test_step_exchange_cpu.py)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = mp.Manager().dict()
    mp.spawn(_rccl_worker, args=(1, port, out), nprocs=1, join=True)
    ref, got, bucketed, loss2 = out[0]
    for a, b, c in zip(ref, got, bucketed):
        assert torch.equal(a, b) and torch.equal(a, c)
    torch.testing.assert_close(loss2, torch.tensor([0.5, 2.0]))


def test_backward_wall_batches_equal_single_batch(monkeypatch):
    """The backward's wall-point batches (bounded dL/drho buffer, NLOSGR_DRHO_MB) give the gradients of
    a single batch: 3 batches vs 1 (summation order of the batch partials differs: rel 1e-5)."""
    from nlosgr import features_flat
    from nlosgr.render import render_backward, render_forward
    dev = torch.device("cuda:0")
    scene, model, geo, cfg, target = _scene_model(dev, ng=1500)
    args = (model._mu.detach(), model._scaling.detach(), model._rotation.detach(), model._opacity.detach(),
            features_flat(model).detach().contiguous())
    hist, _ = render_forward(*args, geo, cfg)
    grad = torch.randn_like(hist)
    ref = render_backward(*args, geo, cfg, grad_hist=grad)
    # 1500 Gaussians x 4 B x 11 wall points per batch: 30 wall points -> 3 batches
    from nlosgr import _lib
    with _lib.batch_budgets(drho_mb=1500 * 4 * 11 / 1048576.0):
        got = render_backward(*args, geo, cfg, grad_hist=grad)
    for a, b in zip(got, ref):
        assert _rel(a, b) <= 1e-5
