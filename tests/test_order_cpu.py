"""slab_order (nlosgr.train): the backward's Gaussian order is a permutation, deterministic, groups
Gaussians by depth slab along the axis facing the relay wall, and is the same for every wall band
of a row-interleaved shard (the bucketed all-reduce relies on it)."""
import torch

from conftest import ROOT  # noqa: F401


def test_slab_order_permutation_and_bands():
    from nlosgr.distributed import wall_rows
    from nlosgr.geometry import relay_wall_grid
    from nlosgr.model import GaussianParams
    from nlosgr.train import slab_order
    m = GaussianParams.synthetic(5000, 3, preset="cuda", device="cpu", seed=4)
    mu = m._mu.detach()
    walls = relay_wall_grid(32, 32)
    perm = slab_order(mu, walls)
    assert torch.equal(torch.sort(perm).values, torch.arange(5000))
    assert torch.equal(perm, slab_order(mu, walls))
    # depth (y: the volume sits at y = 0.5 in front of the wall) is non-decreasing in 8 slabs
    y = mu[perm, 1]
    slab = ((y - y.min()) / (y.max() - y.min()) * 8).floor().clamp(max=7)
    assert bool((slab[1:] >= slab[:-1]).all())
    # with a size key (TrainStep: the largest log-scale) the cells keep their order and each cell is
    # sorted by size
    size = m._scaling.detach().max(1).values
    ps = slab_order(mu, walls, size=size)
    assert torch.equal(torch.sort(ps).values, torch.arange(5000))
    ys = mu[ps, 1]
    slab_s = ((ys - y.min()) / (y.max() - y.min()) * 8).floor().clamp(max=7)
    assert bool((slab_s[1:] >= slab_s[:-1]).all())
    lo, hi = mu.min(0).values, mu.max(0).values
    cell = ((mu - lo) / (hi - lo) * torch.tensor([4.0, 8.0, 4.0])).floor().clamp(max=torch.tensor([3.0, 7.0, 3.0]))
    key = (cell[:, 1] * 4 + cell[:, 0]) * 4 + cell[:, 2]      # slab axis y, then x, z
    ks, ss = key[ps], size[ps]
    same = ks[1:] == ks[:-1]
    assert bool((ks[1:] >= ks[:-1]).all()) and bool((ss[1:][same] >= ss[:-1][same]).all())
    for world in (2, 8):
        for r in range(world):
            band = walls[wall_rows(32, 32, r, world)]
            assert torch.equal(slab_order(mu, band), perm)
            assert torch.equal(slab_order(mu, band, size=size), ps)


def test_forward_order_slabs_by_size():
    """The forward's order (TrainStep fwd_order="slab"): 8 depth slabs, each sorted by size."""
    from nlosgr.geometry import relay_wall_grid
    from nlosgr.model import GaussianParams
    from nlosgr.train import slab_order
    m = GaussianParams.synthetic(3000, 3, preset="cuda", device="cpu", seed=9)
    mu, size = m._mu.detach(), m._scaling.detach().max(1).values
    perm = slab_order(mu, relay_wall_grid(16, 16), 8, 1, size=size)
    assert torch.equal(torch.sort(perm).values, torch.arange(3000))
    y = mu[:, 1]
    slab = ((y - y.min()) / (y.max() - y.min()) * 8).floor().clamp(max=7)[perm]
    assert bool((slab[1:] >= slab[:-1]).all())
    s = size[perm]
    same = slab[1:] == slab[:-1]
    assert bool((s[1:][same] >= s[:-1][same]).all())


def _rank_orders(rank, world, port, out):   # mp.start_processes passes the rank first
    import torch.distributed as dist
    from nlosgr.model import GaussianParams
    from nlosgr.train import slab_order, wall_centroid
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        m = GaussianParams.synthetic(4000, 3, preset="cuda", device="cpu", seed=13)   # replicated on every rank
        mu, size = m._mu.detach(), m._scaling.detach().max(1).values
        # two wall bands whose own centroids face the Gaussians along different axes: band 0 lies far
        # to the side (x = -3: centroid(mu) - centroid(band) is largest along x), band 1 sits under
        # the volume (largest along y); the whole wall's centroid picks x for both
        xs = torch.linspace(-3.2, -2.8, 8) if rank == 0 else torch.linspace(-0.1, 0.3, 8)
        zs = torch.linspace(-0.5, 0.5, 8)
        gx, gz = torch.meshgrid(xs, zs, indexing="ij")
        band = torch.stack([gx.reshape(-1), torch.zeros(64), gz.reshape(-1)], 1)
        c = wall_centroid(band)
        old = slab_order(mu, band, size=size)                   # the round-4 rule: the band's own centroid
        new = slab_order(mu, None, size=size, centroid=c)
        new_f = slab_order(mu, None, 8, 1, size=size, centroid=c)
        olds, news, newfs, cs = ([None] * world for _ in range(4))
        dist.all_gather_object(olds, old)
        dist.all_gather_object(news, new)
        dist.all_gather_object(newfs, new_f)
        dist.all_gather_object(cs, c)
        if rank == 0:
            torch.save({"olds": olds, "news": news, "newfs": newfs, "cs": cs}, out)
    finally:
        dist.destroy_process_group()


def test_slab_order_rank_consistent_across_disagreeing_bands(tmp_path):
    """ADVICE r04 / VERDICT r04 item 7: the slab axis comes from the whole wall's all-reduced centroid,
    so two gloo ranks whose bands would pick different axes under the old per-band rule compute the
    same forward and backward permutations (the bucketed all-reduce sums gradient rows in that order)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "orders.pt")
    mp.start_processes(_rank_orders, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    got = torch.load(out, weights_only=True)
    olds, news, newfs, cs = got["olds"], got["news"], got["newfs"], got["cs"]
    assert not torch.equal(olds[0], olds[1]), "the bands must disagree under the per-band rule"
    assert torch.equal(cs[0], cs[1])
    assert torch.equal(news[0], news[1]) and torch.equal(newfs[0], newfs[1])
    assert torch.equal(torch.sort(news[0]).values, torch.arange(4000))
