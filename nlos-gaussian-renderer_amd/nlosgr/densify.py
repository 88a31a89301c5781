"""MCMC density control for GaussianParams + the fused TrainStep's Adam state.

The reference's version (gaussian_model/gaussian_model.py:391-549: relocate_gs, add_new_gs,
_update_params, _sample_alives, replace_tensors_to_optimizer, cat_tensors_to_optimizer) cannot run:
it calls `compute_relocation_cuda` from the un-vendored 3DGS-MCMC extension, `.unsqeeze` (typo) and
`_sample_alives` without `alive_indices` in add_new_gs. This module restates its intended logic
step by step (same sampling calls, clamps, activations and optimizer-state resets), with the
relocation rule of 3DGS-MCMC ("3D Gaussian Splatting as Markov Chain Monte Carlo", eqs. 9-10, as
implemented by its compute_relocation kernel):
    o' = 1 - (1 - o)^(1/N),   s' = s * o / sum_{i=1..N} sum_{k=0..i-1} C(i-1,k) (-1)^k o'^(k+1) / sqrt(k+1)
evaluated here with the equivalent single sum sum_{k=0..N-1} C(N,k+1) (-1)^k o'^(k+1) / sqrt(k+1)
(hockey-stick identity) in float64. Parity unpinned: no runnable reference exists.
"""
import torch

N_MAX = 51   # 3DGS-MCMC's binomial table size (N is clamped to it)


def compute_relocation(opacity_old, scale_old, N):
    """(new_opacity [n], new_scale [n,3]) for Gaussians split into N copies (N >= 1, clamped to N_MAX)."""
    N = N.clamp(1, N_MAX).to(torch.float64)
    o = opacity_old.to(torch.float64)
    o_new = 1.0 - torch.pow(1.0 - o, 1.0 / N)
    k = torch.arange(N_MAX, dtype=torch.float64, device=o.device)                     # k = 0..N_MAX-1
    lg = torch.lgamma(N[:, None] + 1) - torch.lgamma(k[None] + 2) - torch.lgamma(N[:, None] - k[None])
    binom = torch.where(k[None] < N[:, None], torch.exp(lg), torch.zeros_like(lg))     # C(N, k+1)
    terms = binom * torch.where(k.long() % 2 == 0, 1.0, -1.0)[None] / torch.sqrt(k + 1)[None] \
        * torch.pow(o_new[:, None], k[None] + 1)
    denom = terms.sum(dim=1)
    coeff = o / denom
    return o_new.to(opacity_old.dtype), (coeff[:, None] * scale_old.to(torch.float64)).to(scale_old.dtype)


def _sample_alives(probs, num, alive_indices=None):
    """gaussian_model.py:474-480: multinomial draw (with replacement) proportional to opacity and the
    per-index draw counts."""
    probs = probs / (probs.sum() + torch.finfo(torch.float32).eps)
    idx = torch.multinomial(probs, num, replacement=True)
    if alive_indices is not None:
        idx = alive_indices[idx]
    ratio = torch.bincount(idx).unsqueeze(-1)
    return idx, ratio


def _update_params(model, idxs, ratio):
    """gaussian_model.py:462-472."""
    new_o, new_s = compute_relocation(model.get_opacity[idxs, 0].detach(), model.get_scaling[idxs].detach(),
                                      ratio[idxs, 0] + 1)
    new_o = torch.clamp(new_o.unsqueeze(-1), max=1.0 - torch.finfo(torch.float32).eps, min=0.005)
    new_opacity = torch.log(new_o / (1 - new_o))                                     # inverse sigmoid
    new_scaling = torch.log(new_s.reshape(-1, 3))                                    # inverse of exp
    m = model
    return (m._mu[idxs].detach(), m._features_dc[idxs].detach(), m._features_rest[idxs].detach(),
            new_opacity.reshape(m._opacity[idxs].shape), new_scaling, m._rotation[idxs].detach())


NAMES = ("_mu", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")
ADAM_ORDER = ("_mu", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")   # train.GROUPS


def _moments(step):
    """Adam moments of a TrainStep keyed by parameter name, in the parameters' shapes."""
    if step is None:
        return None
    out = {}
    for i, n in enumerate(ADAM_ORDER):
        shape = getattr(step.model, n).shape
        out[n] = (step.adam.exp_avg[i].view(shape), step.adam.exp_avg_sq[i].view(shape))
    return out


@torch.no_grad()
def relocate_gs(model, dead_mask, train_step=None):
    """gaussian_model.py:484-517: move every dead Gaussian onto a live one drawn by opacity, split the
    opacity / scale of the drawn ones, zero their Adam moments (replace_tensors_to_optimizer(inds))."""
    if dead_mask.sum() == 0:
        return
    alive = ~dead_mask
    dead_idx = dead_mask.nonzero(as_tuple=True)[0]
    alive_idx = alive.nonzero(as_tuple=True)[0]
    if alive_idx.shape[0] <= 0:
        return
    probs = model.get_opacity[alive_idx, 0].detach()
    reinit, ratio = _sample_alives(probs, dead_idx.shape[0], alive_idx)
    vals = _update_params(model, reinit, ratio)
    for n, v in zip(NAMES, vals):
        getattr(model, n).data[dead_idx] = v
    model._opacity.data[reinit] = model._opacity.data[dead_idx]
    model._scaling.data[reinit] = model._scaling.data[dead_idx]
    mom = _moments(train_step)
    if mom is not None:
        for m1, m2 in mom.values():
            m1[reinit] = 0
            m2[reinit] = 0


@torch.no_grad()
def add_new_gs(model, cap_max, train_step=None):
    """gaussian_model.py:519-549: grow by 5 % (up to cap_max) with copies of opacity-sampled Gaussians,
    splitting their opacity / scale; new moments are zero and the sources' moments are reset.
    Returns the number added; a TrainStep passed in is rebound to the grown tensors."""
    cur = model._opacity.shape[0]
    target = min(cap_max, int(1.05 * cur))
    num = max(0, target - cur)
    if num <= 0:
        return 0
    probs = model.get_opacity.detach().reshape(-1)
    add_idx, ratio = _sample_alives(probs, num)
    new = _update_params(model, add_idx, ratio)
    model._opacity.data[add_idx] = new[3]
    model._scaling.data[add_idx] = new[4]
    mom = _moments(train_step)
    grown = {}
    for n, v in zip(NAMES, new):
        old = getattr(model, n).data
        grown[n] = torch.cat((old, v.to(old.dtype)), dim=0).contiguous()
    new_mom = None
    if mom is not None:
        new_mom = {}
        for n in NAMES:
            m1, m2 = mom[n]
            z = torch.zeros((num,) + tuple(m1.shape[1:]), dtype=m1.dtype, device=m1.device)
            a1, a2 = torch.cat((m1, z)), torch.cat((m2, z))
            a1[add_idx] = 0
            a2[add_idx] = 0
            new_mom[n] = (a1, a2)
    for n in NAMES:
        setattr(model, n, torch.nn.Parameter(grown[n]))
    if train_step is not None:
        train_step.rebind([new_mom[n][0] for n in ADAM_ORDER], [new_mom[n][1] for n in ADAM_ORDER])
    return num


def prune_dead_mask(model, min_opacity=0.005):
    """main.py:245: dead = opacity <= 0.005."""
    return (model.get_opacity <= min_opacity).reshape(-1)


__all__ = ["compute_relocation", "relocate_gs", "add_new_gs", "prune_dead_mask", "N_MAX"]
