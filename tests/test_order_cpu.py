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
