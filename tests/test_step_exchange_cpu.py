"""Host logic of the fused training step that runs on CPU (no GPU):

* checkpoint interop: the Adam state TrainStep saves (nlosgr.checkpoint) loads into the reference's
  own torch.optim.Adam over reference-shaped parameters (gaussian_model.py:217-242) and that
  optimizer then steps (moments were saved in TrainStep's flattened view shapes);
* the sharded step's exchange (nlosgr.train.allreduce_step) on world_size-2 gloo
  ranks: summed band gradients and the global (MSE, equal_loss) equal the single-process
  whole-volume values, including a rank whose target band is all zero.
"""
import os
import socket
from types import SimpleNamespace

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT  # noqa: F401  (sys.path setup)


def _ref_params(ng, K):
    g = torch.Generator().manual_seed(4)
    r = lambda *s: torch.randn(*s, generator=g)
    return {"mu": r(ng, 3), "features_dc": r(ng, 1, 1), "features_rest": r(ng, K - 1, 1), "opacity": r(ng, 1),
            "scaling": r(ng, 3), "rotation": r(ng, 4)}


def _fake_step(params, steps=3):
    """Stand-in for TrainStep (which needs a GPU): the flattened group tensors TrainStep keeps."""
    from nlosgr.train import TrainStep
    ng = params["mu"].shape[0]
    flat = [params["mu"], params["features_dc"].view(ng, -1), params["features_rest"].view(ng, -1),
            params["opacity"].view(ng), params["scaling"], params["rotation"]]
    g = torch.Generator().manual_seed(9)
    adam = SimpleNamespace(params=flat, exp_avg=[torch.randn(t.shape, generator=g) for t in flat],
                           exp_avg_sq=[torch.rand(t.shape, generator=g) for t in flat],
                           step_count=steps, betas=(0.9, 0.999), eps=1e-15)
    st = SimpleNamespace(adam=adam, iteration=steps, spatial_lr_scale=1.0)
    from nlosgr.train import OptimizationParams
    st.opt = OptimizationParams()
    st.learning_rates = lambda it: TrainStep.learning_rates(st, it)
    return st


@pytest.mark.parametrize("with_step", [True, False])
def test_checkpoint_optimizer_loads_into_reference_adam(tmp_path, with_step):
    from nlosgr.checkpoint import PARAM_KEYS, save_checkpoint
    from nlosgr.model import GaussianParams
    ng, K = 7, 16
    p = _ref_params(ng, K)
    m = GaussianParams(p["mu"], p["scaling"], p["rotation"], p["opacity"], p["features_dc"], p["features_rest"], 3, 3)
    f = tmp_path / "ck.pt"
    save_checkpoint(str(f), m, _fake_step(p) if with_step else None)
    ck = torch.load(str(f), weights_only=True)
    # the reference's training_setup groups (gaussian_model.py:229-236) over reference-shaped params
    leaves = [torch.nn.Parameter(ck[k].clone()) for k in PARAM_KEYS]
    groups = [{"params": [t], "lr": 1e-3, "name": n} for t, n in
              zip(leaves, ["mu", "f_dc", "f_rest", "opacity", "scaling", "rotation"])]
    opt = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
    opt.load_state_dict(ck["optimizer"])          # restore(): load_state_dict(params['optimizer'])
    for t in leaves:
        t.grad = torch.ones_like(t)
    opt.step()                                    # failed on shape mismatch before the fix
    if with_step:
        for i, t in enumerate(leaves):
            assert opt.state[t]["exp_avg"].shape == t.shape
    assert all(torch.isfinite(t).all() for t in leaves)


def test_checkpoint_fresh_state_mu_lr_has_spatial_scale(tmp_path):
    """Without a TrainStep the saved mu group lr is position_lr_init * spatial_lr_scale, as
    training_setup sets it (gaussian_model.py:230); Adam.load_state_dict copies it over the live one."""
    from nlosgr.checkpoint import save_checkpoint
    from nlosgr.model import GaussianParams
    from nlosgr.train import OptimizationParams
    p = _ref_params(5, 16)
    m = GaussianParams(p["mu"], p["scaling"], p["rotation"], p["opacity"], p["features_dc"], p["features_rest"], 3, 3)
    f = tmp_path / "ck.pt"
    save_checkpoint(str(f), m, None, spatial_lr_scale=2.5)
    ck = torch.load(str(f), weights_only=True)
    lr = ck["optimizer"]["param_groups"][0]["lr"]
    assert ck["optimizer"]["param_groups"][0]["name"] == "mu"
    assert abs(lr - OptimizationParams().position_lr_init * 2.5) < 1e-12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _band_inputs(world):
    """Whole-volume hist/target split into `world` bands; band 1's target is all zero."""
    g = torch.Generator().manual_seed(3)
    P, T = 6, 5
    hist = torch.rand(P, T, generator=g)
    target = torch.rand(P, T, generator=g)
    target[3:] = 0.0
    grads = [torch.randn(8, 3, generator=g) for _ in range(world)]
    return hist, target, grads


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nlosgr.train import allreduce_step
        hist, target, grads = _band_inputs(world)
        b = hist.shape[0] // world
        h, t = hist[rank * b:(rank + 1) * b], target[rank * b:(rank + 1) * b]
        d = h - t
        loss4 = torch.stack([(d * d).mean(), (d * d).mean() / (t * t).mean().clamp_min(1e-30),
                             (d * d).sum(), (t * t).sum()])
        gsum, loss2 = allreduce_step([grads[rank], grads[rank][:, :1]], loss4, hist.numel())
        out[rank] = (gsum[0].clone(), gsum[1].clone(), loss2.clone())
    finally:
        dist.destroy_process_group()


def test_allreduce_step_world2_matches_single_process():
    world = 2
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    hist, target, grads = _band_inputs(world)
    d = hist - target
    loss = (d * d).mean()
    eq = loss / (target * target).mean()
    for r in range(world):
        g0, g1, loss2 = out[r]
        torch.testing.assert_close(g0, grads[0] + grads[1])
        torch.testing.assert_close(g1, (grads[0] + grads[1])[:, :1])
        torch.testing.assert_close(loss2[0], loss, rtol=1e-6, atol=0)
        torch.testing.assert_close(loss2[1], eq, rtol=1e-6, atol=0)
        assert torch.isfinite(loss2).all()


def _bucket_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nlosgr.train import BucketedAllReduce, bucket_bounds
        ng, K = 1000, 16
        g = torch.Generator().manual_seed(10 + rank)
        grads = [torch.randn(ng, 3, generator=g), torch.randn(ng, 1, generator=g), torch.randn(ng, K - 1, generator=g),
                 torch.randn(ng, generator=g), torch.randn(ng, 3, generator=g), torch.randn(ng, 4, generator=g)]
        mine = [t.clone() for t in grads]
        bounds = bucket_bounds(ng, 3)
        ex = BucketedAllReduce(grads, bounds, None)
        for b in range(len(bounds)):
            ex.launch(b)          # TrainStep interleaves these with the per-bucket backward
        out[rank] = ([t.clone() for t in ex.finish()], mine, bounds)
    finally:
        dist.destroy_process_group()


def test_bucketed_allreduce_world2():
    """BucketedAllReduce (TrainStep's overlapped exchange) sums every row of all six
    gradient tensors across ranks, bucket by bucket, back into the same tensors."""
    from nlosgr.train import bucket_bounds
    assert bucket_bounds(1000, 3) == [(0, 512), (512, 1000)]
    assert bucket_bounds(100_000, 4)[0] == (0, 25_088) and bucket_bounds(100_000, 4)[-1][1] == 100_000
    assert all(b0 % 256 == 0 for b0, _ in bucket_bounds(123_457, 7))
    world = 2
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_bucket_worker, args=(world, port, out), nprocs=world, join=True)
    summed = [a + b for a, b in zip(out[0][1], out[1][1])]
    for r in range(world):
        got, _, bounds = out[r]
        assert len(bounds) == 2
        for a, b in zip(got, summed):
            torch.testing.assert_close(a, b)
