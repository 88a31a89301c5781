"""Gaussian initialisation on the GPU: random init and space carving with the
reference's names, arguments and random-number calls (gaussian_model/gaussian_utils.py:8-166).

The reference's space carving loops over every wall point in Python, one torch pass over all
voxels each (gaussian_utils.py:88-99). Here the vote is one HIP launch (`nlosgr_carve_votes`,
lane = voxel, wall points streamed through LDS), and the first-bounce detection
(`detect_first_bounces`, :38-49, a double Python loop over the wall) is one vectorised torch pass.
Meshing (`exact_mesh_samping=True`) needs open3d/trimesh, which the reference imports and this
image lacks: it raises.
"""
import numpy as np
import torch

from . import _lib


def init_rand_points(args, data_kwargs, margin=0.1, rho_scale=0.1, device="cuda"):
    """gaussian_utils.py:8-32: uniform samples in the volume box shrunk by `margin`, rho ~ U(0, rho_scale)
    (numpy global generator, same calls and order as the reference)."""
    n = args.init_gaussian_num
    rho = np.random.rand(n, 1) * rho_scale
    pmin, pmax = data_kwargs["pmin"], data_kwargs["pmax"]
    pmin_c, pmax_c = pmin[:3].cpu().numpy(), pmax[:3].cpu().numpy()
    samples = np.random.rand(n, 3)
    lo = pmin_c + np.abs(pmin_c * margin)
    hi = pmax_c - np.abs(pmax_c * margin)
    return samples * (hi[None] - lo[None]) + lo[None], rho


@torch.no_grad()
def detect_first_bounces(transient, threshold=1e-5):
    """gaussian_utils.py:38-49: per wall pixel (y, x) the first bin b >= 1 with
    transient[b] - transient[b-1] > threshold, 0 if none or if the histogram sums to 0.
    transient [T, H, W] (numpy or torch); returns the same kind, [H, W] float."""
    is_np = isinstance(transient, np.ndarray)
    t = torch.from_numpy(np.ascontiguousarray(transient)) if is_np else transient
    jump = (t[1:] - t[:-1]) > threshold                          # [T-1, H, W], fp32 differences as in numpy
    has = jump.any(dim=0) & (t.sum(dim=0, dtype=torch.float64) != 0)
    first = jump.to(torch.int8).argmax(dim=0) + 1                 # first True (argmax of a 0/1 array)
    out = torch.where(has, first, torch.zeros_like(first)).to(torch.float64 if is_np else torch.float32)
    return out.numpy() if is_np else out


def carve_votes(coords, walls, radius):
    """votes [N] int32: number of first-bounce spheres (walls [M,3], radius [M]) each voxel of
    coords [N,3] lies outside of (radius <= 0 skipped) — one nlosgr_carve_votes launch."""
    lib = _lib.load()
    for t in (coords, walls, radius):
        if not t.is_cuda or t.dtype != torch.float32:
            raise RuntimeError("nlosgr: carve_votes needs float32 GPU tensors (no CPU fallback)")
    coords, walls, radius = coords.contiguous(), walls.contiguous(), radius.contiguous()
    votes = torch.empty(coords.shape[0], dtype=torch.int32, device=coords.device)
    _lib.check(lib.nlosgr_carve_votes(_lib.ptr(coords), coords.shape[0], _lib.ptr(walls), _lib.ptr(radius),
                                      walls.shape[0], _lib.ptr(votes), _lib.stream_handle(coords.device)))
    return votes


@torch.no_grad()
def space_carving(args, data_kwargs):
    """gaussian_utils.py:52-122: voxels of a carving_volume_size^3 grid over the hidden volume that lie
    outside more than space_carving_ratio x max first-bounce spheres; returns their world coordinates
    [Nt, 3] (voxel order of the reference's meshgrid('ij'))."""
    start, threshold = 0, 1e-5      # the reference's only configured scene (zaragoza_bunny, :70-74)
    grid = data_kwargs["camera_grid_positions"]                       # [3, MN]
    device = grid.device
    volume_position = data_kwargs["volume_position"]
    volume_size = data_kwargs["volume_size"]
    c, deltaT = data_kwargs["c"], data_kwargs["deltaT"]
    walls = (grid - volume_position[:, None]).t().contiguous().float()   # shifted origin, [MN, 3]
    nlos = data_kwargs["nlos_data"]
    radii = start + detect_first_bounces(nlos[start:].float(), threshold=threshold).double()
    radii = (radii * c * deltaT).reshape(-1)
    n = args.carving_volume_size
    axis = np.linspace(-volume_size / 2, volume_size / 2, n)
    coords = np.stack(np.meshgrid(axis, axis, axis, indexing="ij"), -1).reshape(-1, 3)
    coords = torch.from_numpy(coords.astype(np.float32)).to(device)
    # the reference compares fp32 distances with the python-float radius cast to fp32
    votes = carve_votes(coords, walls, radii.to(device=device, dtype=torch.float32))
    thr = votes.max().item() * args.space_carving_ratio
    keep = votes > thr
    return coords[torch.nonzero(keep, as_tuple=True)[0]] + volume_position[None]


def sample_from_feasible_space_jittering(args, data_kwargs, margin=0.1, rho_scale=0.1, device="cuda",
                                         exact_mesh_samping=False):
    """gaussian_utils.py:124-166: init_gaussian_num carved voxels drawn with torch.randint and jittered
    by up to half a grid spacing (torch.rand_like), rho ~ U(0, rho_scale) (numpy) — same calls."""
    n = args.init_gaussian_num
    rho = np.random.rand(n, 1) * rho_scale
    coords2 = space_carving(args, data_kwargs)
    if exact_mesh_samping:
        raise NotImplementedError("nlosgr: mesh-based sampling needs open3d / trimesh (absent)")
    pmin, pmax = data_kwargs["pmin"], data_kwargs["pmax"]
    spacing = ((pmax - pmin) / (args.carving_volume_size - 1))[:3]
    half = spacing / 2.0
    idx = torch.randint(0, coords2.shape[0], (n,), device=coords2.device)
    base = coords2[idx]
    return base + (torch.rand_like(base) - 0.5) * 2 * half[None], rho
