"""nlosgr — MI355X-native transient 3D-Gaussian NLOS renderer (hand-written HIP for gfx950).

Layers:
    nlosgr._lib            ctypes binding of the C ABI (include/nlosgr.h, libnlosgr.so)
    nlosgr.render          RenderFn: differentiable batched render (hist [P,T], optional per-ray)
    nlosgr.geometry        batched spherical sampling tables (spherical_sample_histogram for P walls)
    nlosgr.nlos_helpers    drop-in for the reference's nlos_helpers hot path (path T conventions)
    nlosgr.cuda_autograd   drop-in CUDARenderFunction / CUDARenderModule (path C conventions)
    nlosgr.rendering_cuda  drop-in GaussianRendererCUDA / create_cuda_renderer / CUDA_AVAILABLE
    nlosgr.volume          full transient-volume render + MSE loss (the benchmarked step)
    nlosgr.distributed     relay-wall sharding over ranks + one all-reduce of Gaussian gradients
    nlosgr.train           fused training iteration (nlosgr_mse + render fwd/bwd + nlosgr_adam)
    nlosgr.data            Zaragoza capture format, data_shuffle, whole-volume targets / geometry
    nlosgr.checkpoint      reference-keyed checkpoints loadable with weights_only=True
"""
from . import _lib  # noqa: F401
from .geometry import Geometry, build_geometry, relay_wall_grid, volume_box_point  # noqa: F401
from .model import GaussianParams, features_flat  # noqa: F401
from .render import RenderConfig, RenderFn, bboxes, render, render_backward, render_forward  # noqa: F401

__all__ = ["Geometry", "build_geometry", "relay_wall_grid", "volume_box_point", "GaussianParams",
           "features_flat", "RenderConfig", "RenderFn", "render", "render_forward", "render_backward", "bboxes"]
