"""Relay-wall sharding across ranks (one process per GPU) with ONE gradient all-reduce per step.

SURVEY §8e: wall points are independent in the forward (hist[p] depends only on p and all
Gaussians) and the loss is a sum over wall points, so each rank renders a contiguous band of the
H x W wall against a full Gaussian replica and the Gaussian gradients are the SUM of the
per-band partials.  The only exchange is an all_reduce(SUM) of one packed fp32 buffer
[Ng x 27] = (mu 3, scaling 3, rotation 4, opacity 1, features 16) — RCCL ("nccl" backend) on
MI355X, gloo on CPU.  The reference has no multi-GPU path at all; its
single-process step is compute_loss + backward (nlos_helpers.py:280-346, main.py:198-254).

The render function is injectable (`render_fn(model, geo_shard) -> hist [P_shard, T]`) so the
sharding/reduction logic can be exercised on CPU ranks; the default is the HIP render.
"""
import torch
import torch.distributed as dist

from .volume import render_volume


def wall_band(nwall, rank, world):
    """Contiguous [a, b) band of wall points for `rank`: equal counts (±1), SURVEY §8e."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("nlosgr: bad rank/world")
    q, r = divmod(nwall, world)
    a = rank * q + min(rank, r)
    return a, a + q + (1 if rank < r else 0)


def wall_rows(H, W, rank, world, device=None):
    """Row-interleaved shard of an H x W wall for `rank`: wall rows rank, rank + world, ... (row-major
    wall-point indices, int64).  Every rank gets whole wall rows spread over the wall, so the
    per-rank work is balanced (a contiguous band near the wall's centre sees more of the scene than
    one at its edge: up to 1.07x the mean for C5's eight bands); counts differ by at most one row."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("nlosgr: bad rank/world")
    rows = torch.arange(rank, H, world, dtype=torch.int64) if rank < H else torch.zeros(0, dtype=torch.int64)
    idx = (rows.view(-1, 1) * W + torch.arange(W, dtype=torch.int64).view(1, -1)).reshape(-1)
    return idx.to(device) if device is not None else idx


def pack_grads(params):
    """Flatten the .grad of every parameter (zeros where missing) into one contiguous buffer."""
    flat = [(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in params]
    return torch.cat(flat)


def unpack_grads(params, flat):
    off = 0
    for p in params:
        n = p.numel()
        g = flat[off:off + n].view_as(p)
        if p.grad is None:
            p.grad = g.clone()
        else:
            p.grad.copy_(g)
        off += n


def all_reduce_grads(params, group=None):
    """One all_reduce(SUM) of the packed gradient buffer (no-op when not initialised / world 1)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    flat = pack_grads(params)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    unpack_grads(params, flat)


class ShardedVolume:
    """This rank's band of one transient volume: geometry slice + target slice.

    loss = sum over the band of (hist - target)^2 / (P_total * T), so the SUM over ranks of the
    band losses (and of their gradients) equals the single-process volume MSE (volume_loss).
    """

    def __init__(self, geo, target, rank=None, world=None, group=None):
        if rank is None:
            rank = dist.get_rank(group) if dist.is_initialized() else 0
        if world is None:
            world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank, self.world, self.group = rank, world, group
        self.a, self.b = wall_band(geo.nwall, rank, world)
        self.geo = geo.slice(self.a, self.b)
        self.target = target[self.a:self.b]
        self.norm = float(geo.nwall * target.shape[-1])

    def loss(self, model, cfg, render_fn=None):
        hist = render_fn(model, self.geo) if render_fn is not None else render_volume(model, self.geo, cfg)
        d = hist - self.target
        return (d * d).sum() / self.norm

    def step(self, model, cfg, render_fn=None):
        """Forward + band loss + backward + gradient all-reduce.  Returns the GLOBAL loss."""
        params = list(model.parameters())
        for p in params:
            p.grad = None
        loss = self.loss(model, cfg, render_fn)
        loss.backward()
        all_reduce_grads(params, self.group)
        total = loss.detach().clone()
        if dist.is_initialized() and self.world > 1:
            dist.all_reduce(total, op=dist.ReduceOp.SUM, group=self.group)
        return total
