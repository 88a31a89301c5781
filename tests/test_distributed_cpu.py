"""Relay-wall sharding + packed gradient all-reduce on CPU ranks (gloo, world_size 2).

The HIP render is replaced by the CPU oracle through ShardedVolume's render_fn hook, so this
checks the partitioning and reduction logic: the sum over ranks of the band losses/gradients
must equal the single-process full-volume MSE and its gradients.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT  # noqa: F401  (sys.path setup)

NG, DEG, NS, T, H, W = 12, 2, 4, 16, 3, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Model:
    def __init__(self, P):
        self.P = P

    def parameters(self):
        return self.P.leaves()


def _setup():
    from nlosgr.geometry import build_geometry, relay_wall_grid, volume_box_point
    from nlosgr.model import GaussianParams
    from oracle import torch_ref as R
    c, deltaT = 1.0, 1.28 / T
    start, end = T // 8, T // 8 + T
    m = GaussianParams.synthetic(NG, DEG, preset="torch", device="cpu", seed=11)
    P = R.Params(m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
                 m._features_dc.detach(), m._features_rest.detach(), DEG)
    walls = relay_wall_grid(H, W)
    box = volume_box_point((0.0, 0.5, 0.0), 0.5, "cpu")
    geo = build_geometry(walls, box, NS, start, end, c, deltaT, 0.5, "torch", "noocl")
    target = torch.rand(H * W, T, generator=torch.Generator().manual_seed(2)) * 1e-3

    def render_fn(model, g):
        return R.render_volume(model.P, g.wall, box, 0.5, NS, start, end, c, deltaT, preset="torch", mode="noocl")

    return P, geo, target, render_fn


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nlosgr.distributed import ShardedVolume
        P, geo, target, render_fn = _setup()
        sv = ShardedVolume(geo, target)
        loss = sv.step(_Model(P), cfg=None, render_fn=render_fn)
        if rank == 0:
            torch.save({"loss": loss, "grads": [p.grad.clone() for p in P.leaves()], "band": (sv.a, sv.b)}, out)
    finally:
        dist.destroy_process_group()


def test_wall_band_partition():
    from nlosgr.distributed import wall_band
    for n in (0, 1, 7, 64, 16384):
        for world in (1, 2, 3, 8):
            bands = [wall_band(n, r, world) for r in range(world)]
            assert bands[0][0] == 0 and bands[-1][1] == n
            assert all(bands[i][1] == bands[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in bands]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        wall_band(4, 2, 2)


def test_wall_rows_partition():
    """Row-interleaved shards (bench.py's N-rank split): every wall point exactly once, whole rows,
    row counts within one of each other."""
    from nlosgr.distributed import wall_rows
    for H, W in ((1, 1), (7, 3), (128, 128), (256, 256)):
        for world in (1, 2, 3, 8):
            parts = [wall_rows(H, W, r, world) for r in range(world)]
            allidx = torch.cat(parts).sort().values
            assert torch.equal(allidx, torch.arange(H * W))
            assert all(p.numel() % W == 0 for p in parts)
            rows = [p.numel() // W for p in parts]
            assert max(rows) - min(rows) <= 1
            for r, p in enumerate(parts):
                assert torch.equal(p.view(-1, W)[:, 0] // W, torch.arange(r, max(r, H), world))
    with pytest.raises(ValueError):
        wall_rows(4, 4, 2, 2)


def test_pack_unpack_roundtrip():
    from nlosgr.distributed import pack_grads, unpack_grads
    ps = [torch.zeros(5, 3, requires_grad=True), torch.zeros(5, 1, 1, requires_grad=True)]
    ps[0].grad = torch.arange(15.0).view(5, 3)
    flat = pack_grads(ps)
    assert flat.shape == (20,) and torch.equal(flat[15:], torch.zeros(5))
    unpack_grads(ps, flat * 2)
    assert torch.equal(ps[0].grad, 2 * torch.arange(15.0).view(5, 3))
    assert torch.equal(ps[1].grad, torch.zeros(5, 1, 1))


def test_sharded_step_matches_single_process(tmp_path):
    out = str(tmp_path / "rank0.pt")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    got = torch.load(out, weights_only=True)
    assert got["band"] == (0, 3)
    # single process reference: full-volume MSE (volume_loss) and its gradients
    P, geo, target, render_fn = _setup()
    hist = render_fn(_Model(P), geo)
    loss = ((hist - target) ** 2).mean()
    loss.backward()
    torch.testing.assert_close(got["loss"], loss.detach(), rtol=1e-6, atol=0)
    for g, p in zip(got["grads"], P.leaves()):
        torch.testing.assert_close(g, p.grad, rtol=1e-5, atol=1e-12)
