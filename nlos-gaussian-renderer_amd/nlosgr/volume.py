"""Full transient-volume rendering (H x W relay-wall points x T bins in one launch) and the
volume-level training step the benchmark times.

The reference renders one wall point per optimisation step (main.py:198-269,
nlos_helpers.py:302-306); its batched variant is an empty stub (nlos_helpers.py:348-351).
Here the whole relay wall is one batched launch: hist[p, k] for all p, then the MSE of
compute_loss (nlos_helpers.py:323-327) summed over the volume, then one backward launch that
returns the gradients of all six raw parameter tensors.
"""
from dataclasses import dataclass, field

import torch

from .geometry import build_geometry, relay_wall_grid, volume_box_point
from .model import features_flat
from .render import RenderConfig, render


@dataclass
class Scene:
    """Confocal NLOS capture geometry (SURVEY §8d synthetic setup unless overridden)."""
    H: int
    W: int
    T: int
    ns: int = 32
    c: float = 1.0
    deltaT: float = None
    start: int = None
    volume_position: tuple = (0.0, 0.5, 0.0)
    volume_size: float = 0.5
    wall_extent: float = 1.0
    extra: dict = field(default_factory=dict)

    def __post_init__(self):
        if self.deltaT is None:
            self.deltaT = 1.28 / self.T
        if self.start is None:
            self.start = max(1, self.T // 8)

    @property
    def end(self):
        return self.start + self.T

    def walls(self, device):
        return relay_wall_grid(self.H, self.W, self.wall_extent, device)

    def box(self, device):
        return volume_box_point(self.volume_position, self.volume_size, device)

    def geometry(self, device, preset="cuda", mode="noocl", walls=None):
        w = self.walls(device) if walls is None else walls
        return build_geometry(w, self.box(device), self.ns, self.start, self.end, self.c, self.deltaT,
                              self.volume_position[1], preset, mode)


def render_volume(model, geo, cfg):
    """hist [P, T] (differentiable w.r.t. the six raw parameter tensors)."""
    hist, _ = render(model._mu, model._scaling, model._rotation, model._opacity, features_flat(model), geo, cfg,
                     want_hist=True, want_rays=False)
    return hist


def volume_loss(hist, target, reduction="mean"):
    """MSE of compute_loss (nlos_helpers.py:325) over every (wall point, bin) of the volume."""
    d = hist - target
    return (d * d).mean() if reduction == "mean" else (d * d).sum()


def make_config(model, scene, preset="cuda", mode="noocl", cutoff=0.0, scaling_modifier=1.0, selection="support"):
    return RenderConfig(preset=preset, mode=mode, sh_degree=int(model.active_sh_degree),
                        scaling_modifier=scaling_modifier, cutoff=cutoff, c_deltaT=scene.c * scene.deltaT,
                        ray_scale=(scene.c * scene.deltaT if (preset == "cuda" and mode in ("noocl", "binint")) else 1.0),
                        selection=selection)


def train_step(model, geo, cfg, target, loss_scale=1.0):
    """Forward + MSE + backward; leaves .grad on the six parameters and returns the loss."""
    for p in model.parameters():
        p.grad = None
    hist = render_volume(model, geo, cfg)
    loss = volume_loss(hist, target) * loss_scale
    loss.backward()
    return loss.detach()
