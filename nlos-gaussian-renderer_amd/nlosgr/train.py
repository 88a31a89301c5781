"""Fused on-device training step over the whole transient volume.

The reference's training iteration (main.py:198-254 learn_one_iter) is, per wall point:
update_learning_rate -> zero_grad -> compute_loss (render + MSE vs gt_times * data,
nlos_helpers.py:280-346) -> backward -> optimizer.step (torch.optim.Adam over six parameter
groups, gaussian_model.py:223-242) -> oneupSHdegree (main.py:240-241).  TrainStep runs the same
iteration for a whole volume (or this rank's band of it) with every piece on the device and no
host synchronisation inside the step:

    render_forward (HIP, records the ray cache)  ->  nlosgr_mse (loss, equal_loss, dL/dhist)
    ->  render_backward (HIP, walks the ray cache)  ->  [one packed all-reduce when sharded]
    ->  nlosgr_adam (all six groups in one launch; position lr from get_expon_lr_func)

The returned loss is a device tensor; reading it is the caller's choice (and its only sync).
"""
import math
import os
from dataclasses import dataclass, replace

import torch
import torch.distributed as dist

from . import _lib
from .model import features_flat
from .render import render_backward, render_forward, tile_rows_bytes, use_ray_cache

# occlusion mode: wall points per fused forward/MSE/backward batch are sized so that the batch's row
# cache (the forward's (D, W) rows, reloaded by the backward) stays within this budget
OCCL_BATCH_BYTES = int(float(os.environ.get("NLOSGR_OCCL_BATCH_GB", "8")) * 2 ** 30)

GROUPS = ("mu", "f_dc", "f_rest", "opacity", "scaling", "rotation")   # gaussian_model.py:229-236


def expon_lr(step, lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """get_expon_lr_func(...)(step) (gaussian_utils.py:223-256): log-linear decay from lr_init to
    lr_final over max_steps, optionally eased in over lr_delay_steps."""
    if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
        return 0.0
    if lr_delay_steps > 0:
        delay_rate = lr_delay_mult + (1 - lr_delay_mult) * math.sin(0.5 * math.pi * min(max(step / lr_delay_steps,
                                                                                           0.0), 1.0))
    else:
        delay_rate = 1.0
    t = min(max(step / max_steps, 0.0), 1.0)
    return delay_rate * math.exp(math.log(lr_init) * (1 - t) + math.log(lr_final) * t)


@dataclass
class OptimizationParams:
    """The optimiser fields of configs/default.py:59-69 (OptimizationParams) the step uses."""
    position_lr_init: float = 0.00016
    position_lr_final: float = 0.0000016
    position_lr_delay_mult: float = 0.01
    position_lr_max_steps: int = 50_000
    feature_lr: float = 0.0025
    opacity_lr: float = 0.025
    scaling_lr: float = 0.005
    rotation_lr: float = 0.001
    regularization: bool = False     # configs/default.py:88-90, applied in learn_one_iter (main.py:204-208)
    scale_reg: float = 0.01
    opacity_reg: float = 0.01


def mse(hist, target, gt_times=1.0, grad_scale=1.0, want_grad=True, raw=False):
    """(loss2, grad): loss2 = device [2] = (MSE, equal_loss) of compute_loss
    (nlos_helpers.py:323-327) against gt_times * target; grad = grad_scale * dMSE/dhist.
    raw=True returns the device [4] (MSE, equal_loss, sum d^2, sum (gt target)^2)."""
    lib = _lib.load()
    dev = hist.device
    h = hist.detach().contiguous()
    t = target.detach().contiguous()
    if h.shape != t.shape or h.dtype != torch.float32 or t.dtype != torch.float32:
        raise ValueError("nlosgr: hist and target must be float32 tensors of one shape")
    ws = torch.empty(lib.nlosgr_mse_workspace_bytes() // 4, dtype=torch.float32, device=dev)
    out = torch.empty(4, dtype=torch.float32, device=dev)
    grad = torch.empty_like(h) if want_grad else None
    _lib.check(lib.nlosgr_mse(_lib.ptr(h), _lib.ptr(t), float(gt_times), h.numel(), float(grad_scale),
                              _lib.ptr(grad), _lib.ptr(ws), _lib.ptr(out), _lib.stream_handle(dev)))
    return (out if raw else out[:2]), grad


def pack_grads(grads):
    """One contiguous fp32 buffer of the six gradient tensors (group order) and the split views."""
    flat = torch.cat([g.reshape(-1) for g in grads])
    views, off = [], 0
    for g in grads:
        views.append(flat[off:off + g.numel()].view(g.shape))
        off += g.numel()
    return flat, views


def allreduce_step(grads, loss4, n_total, group=None, async_op=False):
    """The exchange of one sharded training step: ONE all-reduce(SUM) of the packed
    gradient buffer plus one of the two raw loss sums, then the global (MSE, equal_loss) of the
    whole volume = (sum d^2 / n_total, sum d^2 / sum (gt t)^2) — exact for any band split, and
    finite when a band's target is all zero.  Returns (grads, loss2) (or the work handles first when
    async_op).  The caller's band gradients must already carry the n_local / n_total scale."""
    flat, views = pack_grads(grads)
    sums = loss4[2:4].clone()
    w1 = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
    w2 = dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group, async_op=async_op)

    def finish():
        se, st = sums[0], sums[1]
        loss = se / float(n_total)
        eq = torch.where(st > 0, se / st, torch.zeros_like(se))
        return views, torch.stack([loss, eq])
    if async_op:
        return (w1, w2), finish
    return finish()


def wall_centroid(wall, group=None, reduce=True):
    """Centroid of the WHOLE relay wall.  With a wall shard per rank (world > 1) the sum and count of
    every rank's wall points are all-reduced over `group`, so every rank gets the same centroid
    (slab_order's axis must not depend on which band a rank renders).  reduce=False: this wall only,
    no collective (a caller whose group has one rank must not all-reduce over the default group)."""
    w = wall.detach().reshape(-1, 3).double()
    s = torch.cat([w.sum(0), torch.tensor([float(w.shape[0])], dtype=torch.float64, device=w.device)])
    if reduce and dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(s, op=dist.ReduceOp.SUM, group=group)
    return (s[:3] / s[3].clamp_min(1.0)).float()


def slab_order(mu, wall, slabs=8, cells=4, size=None, size_buckets=0, centroid=None):
    """Permutation of the Gaussians for the backward: sorted by cell of a slabs x cells x cells grid over
    their bounding box, slab (the coordinate axis along which the Gaussians lie in front of the relay
    wall: the largest component of centroid(mu) - centroid(wall)) major, then the other two axes in
    order, and inside a cell by `size` (ascending; TrainStep passes the largest log-scale).  The
    backward's workgroups own 64 consecutive Gaussians: spatially compact blocks of alike size have
    alike candidate boxes and ray counts at every wall point, so the block's enumeration and drain end
    together instead of waiting for its largest pair.  C3 backward (same box, scripts/env_ab.sh):
    given order 951 ms, 16x8 cells 937, 8x4 cells + size 887; size-quantile-major buckets 911
    (`size_buckets`).  Any order gives the same gradients up to fp32 summation order.
    Rank-consistent: `centroid` (wall_centroid: the whole wall's, all-reduced) replaces the centroid of
    `wall`, so the ranks of a wall shard, which hold the same Gaussians, compute the same permutation
    whatever their bands (the bucketed all-reduce sums gradient rows in this order)."""
    with torch.no_grad():
        wc = centroid.to(mu.device, mu.dtype) if centroid is not None else wall.reshape(-1, 3).mean(0)
        d = mu.mean(0) - wc
        k = int(torch.argmax(d.abs()))
        axes = [k] + [i for i in range(3) if i != k]
        q = mu[:, axes]
        lo, hi = q.min(0).values, q.max(0).values
        n = torch.tensor([slabs, cells, cells], device=mu.device, dtype=q.dtype)
        cell = ((q - lo) / (hi - lo).clamp_min(1e-12) * n).floor().clamp(max=n - 1).long()
        key = (cell[:, 0] * cells + cell[:, 1]) * cells + cell[:, 2]
        if size is None:
            return torch.argsort(key, stable=True)
        if size_buckets:                                     # size-quantile bucket major, then cell
            rank = torch.empty_like(key)
            rank[torch.argsort(size, stable=True)] = torch.arange(key.numel(), device=key.device)
            b = rank * size_buckets // key.numel()
            return torch.argsort(b * (slabs * cells * cells) + key, stable=True)
        by_size = torch.argsort(size, stable=True)          # within a cell: ascending size
        return by_size[torch.argsort(key[by_size], stable=True)]


def bucket_bounds(ng, nbuckets):
    """Gaussian ranges [g0, g1) of the bucketed gradient exchange; g0 is a multiple of 256 (the
    backward's Gaussian-block granularity, nlosgr_options.g_begin)."""
    if nbuckets <= 1 or ng <= 256:
        return [(0, ng)]
    step = ((ng + nbuckets - 1) // nbuckets + 255) // 256 * 256
    return [(g0, min(ng, g0 + step)) for g0 in range(0, ng, step)]


class BucketedAllReduce:
    """SURVEY §8e overlap: the six gradient tensors (GROUPS order, rows = Gaussians) are exchanged in
    Gaussian buckets.  launch(b) packs rows [g0, g1) of every tensor into one contiguous buffer on the
    current stream and issues an asynchronous all-reduce(SUM) of it (RCCL orders it after the work
    already queued, so it runs while the next bucket is differentiated); finish() waits for all
    buckets and writes the sums back into the tensors."""

    def __init__(self, grads, bounds, group=None):
        self.grads, self.bounds, self.group = grads, bounds, group
        self.works, self.bufs = [], []

    def launch(self, b):
        g0, g1 = self.bounds[b]
        buf = torch.cat([g[g0:g1].reshape(-1) for g in self.grads])
        self.bufs.append((b, buf))
        self.works.append(dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def finish(self):
        for w in self.works:
            w.wait()
        for b, buf in self.bufs:
            g0, g1 = self.bounds[b]
            off = 0
            for g in self.grads:
                n = (g1 - g0) * (g[0].numel() if g.dim() > 1 else 1)
                g[g0:g1].copy_(buf[off:off + n].view_as(g[g0:g1]))
                off += n
        self.works, self.bufs = [], []
        return self.grads


class Adam:
    """torch.optim.Adam (no weight decay / amsgrad) on the device for a fixed list of contiguous
    fp32 tensors, one launch per step (nlosgr_adam)."""

    def __init__(self, params, betas=(0.9, 0.999), eps=1e-15):
        if not 1 <= len(params) <= _lib.ADAM_MAX_GROUPS:
            raise ValueError("nlosgr: 1..8 parameter groups")
        for p in params:
            if p.dtype != torch.float32 or not p.is_contiguous() or not p.is_cuda:
                raise ValueError("nlosgr: Adam parameters must be contiguous float32 GPU tensors")
        self.params = list(params)
        self.exp_avg = [torch.zeros_like(p) for p in params]
        self.exp_avg_sq = [torch.zeros_like(p) for p in params]
        self.betas, self.eps, self.step_count = betas, eps, 0

    def step(self, grads, lrs):
        lib = _lib.load()
        self.step_count += 1
        gs = []
        arr = (_lib.AdamGroup * len(self.params))()
        for i, (p, g, lr) in enumerate(zip(self.params, grads, lrs)):
            g = g.detach().reshape(p.shape).contiguous()
            gs.append(g)   # keep alive until the launch is enqueued
            arr[i] = _lib.AdamGroup(_lib.ptr(p), _lib.ptr(g), _lib.ptr(self.exp_avg[i]),
                                    _lib.ptr(self.exp_avg_sq[i]), p.numel(), float(lr))
        _lib.check(lib.nlosgr_adam(arr, len(self.params), self.step_count, float(self.betas[0]),
                                   float(self.betas[1]), float(self.eps), _lib.stream_handle(self.params[0].device)))


class TrainStep:
    """One fused training iteration per call (see module docstring).

    model   : GaussianModel-like (raw tensors _mu, _scaling, _rotation, _opacity, _features_dc,
              _features_rest and active_sh_degree); updated in place.
    geo     : nlosgr Geometry of the wall points this process renders (the whole wall, or this
              rank's band from nlosgr.distributed.wall_band).
    target  : [P, T] measured histograms of those wall points (before gt_times).
    nwall_total : wall points of the whole volume (the MSE is normalised over the whole volume and
              the band gradients / losses are summed over ranks).
    """

    def __init__(self, model, geo, cfg, target, gt_times=1.0, opt=None, spatial_lr_scale=1.0, nwall_total=None,
                 group=None, sh_schedule=False, events=None, buckets=4, keep_grads=False, bwd_order="slab",
                 fwd_order="slab"):
        self.model, self.geo, self.cfg = model, geo, cfg
        # backward / forward Gaussian orders (slab_order; None = as stored)
        self.bwd_order = bwd_order
        self.fwd_order = fwd_order
        self.keep_grads = keep_grads   # tests: keep the last step's (all-reduced) gradients in self.grads,
        self.grads = None              # its forward volume in self.hist and its dL/dhist in self.grad_hist
        self.hist = self.grad_hist = None
        self.target = target.detach().float().contiguous()
        self.gt_times = float(gt_times)
        self.opt = opt or OptimizationParams()
        self.spatial_lr_scale = float(spatial_lr_scale)
        self.group = group
        self.world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
        self.n_local = geo.nwall * geo.nr
        if nwall_total is None and self.world > 1:
            # every rank renders its own band: the MSE normalises over the whole volume
            t = torch.tensor([float(geo.nwall)], device=model._mu.device)
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
            nwall_total = int(t.item())
        self.n_total = (nwall_total if nwall_total is not None else geo.nwall) * geo.nr
        self.sh_schedule = sh_schedule
        self.events = events      # optional {"fwd": (start, end), "bwd": (start, end)} HIP events (bench timing)
        self.buckets = int(buckets)   # gradient all-reduce buckets overlapped with the backward (world > 1)
        self.iteration = 0
        self._batch_events = []
        self._occl_plan = None           # occlusion mode: wall-point batches, planned at the first step
        # the slab orders' axis comes from the whole wall's centroid (the same on every rank)
        self.wall_c = wall_centroid(geo.wall, group, reduce=self.world > 1)
        ng = model._mu.shape[0]
        self._tensors = [model._mu.data, model._features_dc.data.view(ng, -1), model._features_rest.data.view(ng, -1),
                         model._opacity.data.view(ng), model._scaling.data, model._rotation.data]
        self.adam = Adam(self._tensors, eps=1e-15)

    def rebind(self, exp_avg=None, exp_avg_sq=None):
        """Re-point the step at the model's (possibly resized) parameter tensors after density control
        (nlosgr.densify); the Adam moments are replaced by the given lists (group order of GROUPS) and
        the step count is kept."""
        m = self.model
        ng = m._mu.shape[0]
        self._occl_plan = None
        self._tensors = [m._mu.data, m._features_dc.data.view(ng, -1), m._features_rest.data.view(ng, -1),
                         m._opacity.data.view(ng), m._scaling.data, m._rotation.data]
        step_count = self.adam.step_count
        self.adam = Adam(self._tensors, betas=self.adam.betas, eps=self.adam.eps)
        self.adam.step_count = step_count
        if exp_avg is not None:
            for i, (a, b) in enumerate(zip(exp_avg, exp_avg_sq)):
                self.adam.exp_avg[i].copy_(a.reshape(self._tensors[i].shape))
                self.adam.exp_avg_sq[i].copy_(b.reshape(self._tensors[i].shape))

    def learning_rates(self, iteration):
        o = self.opt
        mu_lr = expon_lr(iteration, o.position_lr_init * self.spatial_lr_scale,
                         o.position_lr_final * self.spatial_lr_scale, lr_delay_mult=o.position_lr_delay_mult,
                         max_steps=o.position_lr_max_steps)     # update_learning_rate, gaussian_model.py:244-249
        return [mu_lr, o.feature_lr, o.feature_lr / 20.0, o.opacity_lr, o.scaling_lr, o.rotation_lr]

    def occl_batches(self):
        """Wall-point ranges [p0, p1) of the occlusion mode's fused batches (row cache <= OCCL_BATCH_BYTES).
        Planned once (and again after rebind()), so the batch split, hence the summation order and the
        cached/recompute choice, is the same every step."""
        if self._occl_plan is not None:
            return self._occl_plan
        P = self.geo.nwall
        per = max(1, tile_rows_bytes(self.geo) // max(1, P))
        budget = OCCL_BATCH_BYTES
        if self.geo.wall.is_cuda:
            # at most half the free device memory (the batch's row cache is allocated per batch), counting
            # the blocks the caching allocator holds but no tensor uses; when not even one wall point's
            # rows fit, the backward recomputes the forward sweep instead
            dev = self.geo.wall.device
            free, _ = torch.cuda.mem_get_info(dev)
            free += torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
            budget = min(budget, free // 2)
        self._occl_cache = budget >= per
        nb = max(1, budget // per)
        self._occl_plan = [(p0, min(P, p0 + nb)) for p0 in range(0, P, nb)]
        return self._occl_plan

    def phase_ms(self):
        """(forward, backward) milliseconds of the last step from its HIP events (after a synchronize);
        the occlusion mode's batches are summed per phase."""
        ev = self.events
        if self._batch_events:
            f = sum(a.elapsed_time(b) for a, b, _, _ in self._batch_events)
            g = sum(c.elapsed_time(d) for _, _, c, d in self._batch_events)
            return f, g
        return ev["fwd"][0].elapsed_time(ev["fwd"][1]), ev["bwd"][0].elapsed_time(ev["bwd"][1])

    def _occl_step(self, args, cfg):
        """Occlusion compositing (path C's shared transmittance): the wall is rendered in batches of
        wall points; per batch the forward stores its tiles' (D, W) rows, the MSE gradient of the batch
        follows at once (the loss is a sum over wall points) and the backward reloads the rows instead
        of re-running the forward sweep, so the row cache is bounded by the batch (C3: 8 GiB of rows
        per 1024 wall points instead of 128 GiB for the wall).  Returns (grads, loss4)."""
        dev = args[0].device
        stream = torch.cuda.current_stream(dev) if self.events else None
        sums = torch.zeros(2, dtype=torch.float32, device=dev)
        acc = None
        params = args[:5]
        for (p0, p1) in self.occl_batches():
            geo = self.geo.slice(p0, p1) if (p0, p1) != (0, self.geo.nwall) else self.geo
            evs = None
            if self.events:
                evs = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                self._batch_events.append(tuple(evs))
                evs[0].record(stream)
            cached = self._occl_cache
            if cached:
                try:
                    hist, _, ws = render_forward(*params, geo, cfg, True, False, ray_cache=True)
                except torch.cuda.OutOfMemoryError:
                    # the planned row cache did not fit after all (the caching allocator's free blocks
                    # counted in occl_batches may be fragmented): recompute from here on
                    self._occl_cache = cached = False
            if not cached:
                (hist, _), ws = render_forward(*params, geo, cfg, True, False), None
            if evs:
                evs[1].record(stream)
            n_b = geo.nwall * geo.nr
            loss4, grad = mse(hist, self.target[p0:p1], self.gt_times, grad_scale=n_b / self.n_total, raw=True)
            sums += loss4[2:4]
            if evs:
                evs[2].record(stream)
            d = render_backward(*params, geo, cfg, grad_hist=grad, workspace=ws, ray_cache=cached)
            if evs:
                evs[3].record(stream)
            del ws, hist, grad
            acc = list(d) if acc is None else [a.add_(b) for a, b in zip(acc, d)]
        d_mu, d_s, d_q, d_o, d_f = acc
        se, st = sums[0], sums[1]
        loss4 = torch.stack([se / float(self.n_total), torch.where(st > 0, se / st, torch.zeros_like(se)), se, st])
        return [d_mu, d_f[:, :1], d_f[:, 1:], d_o, d_s, d_q], loss4

    def __call__(self, iteration=None):
        it = self.iteration if iteration is None else iteration
        m = self.model
        ng = m._mu.shape[0]
        cfg = replace(self.cfg, sh_degree=int(m.active_sh_degree))
        feats = features_flat(m).detach().contiguous()
        args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), feats, self.geo)
        self._batch_events = []
        if cfg.mode == "occl" and cfg.ray_cache:
            grads, loss4 = self._occl_step(args, cfg)
            loss2 = loss4[:2]
            if self.world > 1:
                grads, loss2 = allreduce_step(grads, loss4, self.n_total, self.group)
            return self._finish(grads, loss2, it)
        cache = use_ray_cache(cfg, self.geo, ng)
        ev = self.events
        stream = torch.cuda.current_stream(m._mu.device) if ev else None
        if ev:
            ev["fwd"][0].record(stream)
        if self.fwd_order == "slab" and not cache and cfg.mode != "occl" and cfg.selection == "support" and ng > 64:
            # (not under path C's AABB selection: its first-256-hits rule depends on the Gaussian order)
            # the forward renders the Gaussians in 8 depth slabs, each sorted by size (largest
            # log-scale): a wave's 64 pairs then have alike candidate boxes and segment lengths, and the
            # slabs keep them spread over the ToF bins (claim collisions).  C3 forward 1086 -> 1050 ms;
            # 4 / 16 / 32 slabs the same, no slabs (size only) 1077, with lateral cells 1101.  The
            # histogram is order-independent up to fp32 summation order.
            fp = slab_order(args[0], None, 8, 1, size=args[1].max(1).values, centroid=self.wall_c)
            out = render_forward(*(tuple(t[fp].contiguous() for t in args[:5]) + (args[5],)), cfg, True, False,
                                 ray_cache=cache)
        else:
            out = render_forward(*args, cfg, True, False, ray_cache=cache)
        if ev:
            ev["fwd"][1].record(stream)
        hist, ws = out[0], (out[2] if cache else None)
        loss4, grad = mse(hist, self.target, self.gt_times, grad_scale=self.n_local / self.n_total, raw=True)
        loss2 = loss4[:2]
        if self.keep_grads:
            self.hist, self.grad_hist = hist, grad
        if ev:
            ev["bwd"][0].record(stream)
        bounds = bucket_bounds(ng, self.buckets) if (self.world > 1 and cfg.mode != "occl"
                                                     and cfg.selection == "support") else [(0, ng)]
        # the backward renders the Gaussians in slab order (not with the ray cache: its records are
        # indexed by the forward's order); its gradients are scattered back below
        perm = None
        if self.bwd_order == "slab" and not cache and cfg.mode != "occl" and cfg.selection == "support" and ng > 64:
            # 8 slabs x 4 x 4 cells, largest log-scale within a cell (grid and key A/B'd in round 4)
            perm = slab_order(args[0], None, 8, 4, size=args[1].max(1).values, centroid=self.wall_c)
            args = tuple(t[perm].contiguous() for t in args[:5]) + (args[5],)

        def unperm(gs):
            if perm is None:
                return gs
            out = []
            for gr in gs:
                o = torch.empty_like(gr)
                o[perm] = gr
                out.append(o)
            return out
        if len(bounds) > 1:
            # bucketed: differentiate Gaussians [g0, g1), then all-reduce that bucket asynchronously
            # while the next bucket's backward runs (SURVEY §8e overlap)
            outs = (torch.empty_like(args[0]), torch.empty_like(args[1]), torch.empty_like(args[2]),
                    torch.empty(ng, device=m._mu.device), torch.empty_like(feats))
            d_mu, d_s, d_q, d_o, d_f = outs
            ex = BucketedAllReduce([d_mu, d_f[:, :1], d_f[:, 1:], d_o, d_s, d_q], bounds, self.group)
            for b, gr in enumerate(bounds):
                render_backward(*args, cfg, grad_hist=grad, workspace=ws, ray_cache=cache, g_range=gr, out=outs)
                ex.launch(b)
            sums = loss4[2:4].clone()
            dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=self.group)
            if ev:
                ev["bwd"][1].record(stream)
            grads = unperm(ex.finish())
            se, st = sums[0], sums[1]
            loss2 = torch.stack([se / float(self.n_total), torch.where(st > 0, se / st, torch.zeros_like(se))])
            del ws
        else:
            d_mu, d_s, d_q, d_o, d_f = unperm(render_backward(*args, cfg, grad_hist=grad, workspace=ws,
                                                              ray_cache=cache))
            if ev:
                ev["bwd"][1].record(stream)
            del ws
            grads = [d_mu, d_f[:, :1], d_f[:, 1:], d_o, d_s, d_q]
            if self.world > 1:
                grads, loss2 = allreduce_step(grads, loss4, self.n_total, self.group)
        return self._finish(grads, loss2, it)

    def _finish(self, grads, loss2, it):
        m = self.model
        if self.opt.regularization:
            # + opacity_reg mean|sigmoid(o)| + scale_reg mean|exp(s)| (main.py:204-208); replicated
            # terms, so added after the all-reduce.  equal_loss stays the render term's (as there).
            o = m._opacity.detach().reshape(-1)
            so = torch.sigmoid(o)
            es = torch.exp(m._scaling.detach())
            grads[3] = grads[3] + (self.opt.opacity_reg / o.numel()) * so * (1.0 - so)
            grads[4] = grads[4] + (self.opt.scale_reg / es.numel()) * es
            reg = self.opt.opacity_reg * so.mean() + self.opt.scale_reg * es.mean()
            loss2 = torch.stack([loss2[0] + reg, loss2[1]])
        if self.keep_grads:
            self.grads = [g.clone() for g in grads]
        self.adam.step(grads, self.learning_rates(it))
        self.iteration = it + 1
        if self.sh_schedule and self.iteration % 1000:   # main.py:240-241 (fires when NOT a multiple)
            m.oneupSHdegree()
        return loss2
