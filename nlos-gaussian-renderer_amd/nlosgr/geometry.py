"""Per-wall-point spherical sampling tables, batched over relay-wall points on the device.

Restates nlos_helpers.py:124-188 (spherical_sample_histogram) for P wall points at once:
angular box of the hidden volume's 8 corners seen from each wall point, torch-linspace
theta / phi grids, shared radial grid r, and the attenuation tables of the two presets
(nlos_helpers.py:216-229 for "torch", gaussian_model/cuda_autograd.py:301-314 for "cuda").
No `.item()` host syncs: everything stays on the device.
"""
import math
from dataclasses import dataclass

import torch


def volume_box_point(volume_position, volume_size, device=None):
    """nlos_helpers.py:107-118 — the 8 corners of the hidden volume in the reference's order."""
    xv, yv, zv = [float(v) for v in volume_position]
    h = volume_size / 2
    x = [xv - h] * 4 + [xv + h] * 4
    y = [yv - h, yv - h, yv + h, yv + h] * 2
    z = [zv - h, zv + h] * 4
    return torch.tensor([x, y, z], dtype=torch.float64).t().contiguous().float().to(device)


def linspace_rows(lo, hi, n):
    """torch.linspace(lo[p], hi[p], n) for every row p (ATen's two-sided formula:
    start + step*i for i < n//2, end - step*(n-1-i) otherwise)."""
    P = lo.shape[0]
    if n == 1:
        return lo.reshape(P, 1).clone()
    lo = lo.float()
    hi = hi.float()
    step = ((hi - lo) / (n - 1)).double()          # fp32 step, as ATen computes it
    i = torch.arange(n, device=lo.device, dtype=torch.float64)
    # ATen evaluates start + step*i with a fused multiply-add: emulate with one rounding from fp64
    fwd = lo.double()[:, None] + step[:, None] * i[None, :]
    bwd = hi.double()[:, None] - step[:, None] * (n - 1 - i)[None, :]
    return torch.where((i < (n // 2))[None, :], fwd, bwd).float()


def angle_ranges(walls, box):
    """min/max of theta = acos(z/r), phi = atan2(y, x) of (corner - wall) over the 8 corners
    (nlos_helpers.py:149-156, cartesian2spherical_torch :87-95).  walls [P,3], box [8,3]."""
    bp = box[None, :, :] - walls[:, None, :]                       # [P,8,3]
    r = torch.linalg.norm(bp, dim=2)
    th = torch.acos(bp[..., 2] / r)
    ph = torch.atan2(bp[..., 1], bp[..., 0])
    return th.min(1).values, th.max(1).values, ph.min(1).values, ph.max(1).values


@dataclass
class Geometry:
    """Device tables consumed by nlosgr_render_fwd/bwd (layout of nlosgr_geometry)."""
    wall: torch.Tensor        # [P,3]
    sin_theta: torch.Tensor   # [P,nt]
    cos_theta: torch.Tensor
    sin_phi: torch.Tensor     # [P,np]
    cos_phi: torch.Tensor
    grid_lin: torch.Tensor    # [P,4]
    hscale: torch.Tensor      # [P]
    r: torch.Tensor           # [nr]
    att: torch.Tensor         # [nr]
    theta: torch.Tensor       # [P,nt]  (kept for the per-ray post-processing of the drop-in API)
    phi: torch.Tensor         # [P,np]
    nt: int
    np: int
    nr: int

    @property
    def nwall(self):
        return self.wall.shape[0]

    def slice(self, a, b):
        """Wall points [a, b) (for sharding the relay wall across ranks)."""
        return Geometry(self.wall[a:b], self.sin_theta[a:b], self.cos_theta[a:b], self.sin_phi[a:b],
                        self.cos_phi[a:b], self.grid_lin[a:b], self.hscale[a:b], self.r, self.att,
                        self.theta[a:b], self.phi[a:b], self.nt, self.np, self.nr)

    def rows(self, idx):
        """Wall points idx (int64, e.g. distributed.wall_rows: the row-interleaved shard bench.py uses)."""
        idx = idx.to(self.wall.device)
        pick = lambda t: t.index_select(0, idx).contiguous()
        return Geometry(pick(self.wall), pick(self.sin_theta), pick(self.cos_theta), pick(self.sin_phi),
                        pick(self.cos_phi), pick(self.grid_lin), pick(self.hscale), self.r, self.att,
                        pick(self.theta), pick(self.phi), self.nt, self.np, self.nr)


def radial_tables(start, end, c, deltaT, preset, device):
    """r_k and the per-bin attenuation.
    torch: r = linspace(start cdT, end cdT, nr) (nlos_helpers.py:169-172), att = 1/dist^2 with
           dist = linspace(I1, I2, nr)*dT*c (:219);  cuda: t = linspace(I1 cdT, I2 cdT, nr),
           att = 1/(t^2+1e-8) (nlos_helpers.py:251-252, cuda_autograd.py:273,308)."""
    nr = end - start
    r_min = start * c * deltaT
    r_max = end * c * deltaT
    I1 = math.floor(r_min / (c * deltaT))
    I2 = math.ceil(r_max / (c * deltaT))
    if preset == "torch":
        r = torch.linspace(r_min, r_max, nr, dtype=torch.float, device=device)
        dist = torch.linspace(I1, I2, nr, dtype=torch.float, device=device) * deltaT * c
        att = 1.0 / (dist ** 2)
    else:
        r = torch.linspace(I1 * c * deltaT, I2 * c * deltaT, nr, dtype=torch.float, device=device)
        att = 1.0 / (r ** 2 + 1e-8)
    return r.contiguous(), att.contiguous(), I1, I2


def geometry_from_ranges(walls, tmin, tmax, pmin, pmax, nt, nphi, r, att, hscale_extra=1.0,
                         theta=None, phi=None):
    """Tables from per-wall-point angular ranges [P] (theta/phi default to the torch linspace
    grids; pass explicit [P,nt]/[P,np] grids to reuse a caller's exact sample values)."""
    theta = linspace_rows(tmin, tmax, nt) if theta is None else theta.float()
    phi = linspace_rows(pmin, pmax, nphi) if phi is None else phi.float()
    step_t = (tmax - tmin) / (nt - 1) if nt > 1 else torch.zeros_like(tmin)
    step_p = (pmax - pmin) / (nphi - 1) if nphi > 1 else torch.zeros_like(pmin)
    grid_lin = torch.stack([tmin, step_t, pmin, step_p], dim=1).float().contiguous()
    # dtheta = (max-min)/Ns (not /(Ns-1)), nlos_helpers.py:163-164; hist *= dtheta*dphi (:229)
    dth = (tmax.double() - tmin.double()) / nt
    dph = (pmax.double() - pmin.double()) / nphi
    hscale = (dth * dph * hscale_extra).float().contiguous()
    return Geometry(walls.float().contiguous(), torch.sin(theta).contiguous(), torch.cos(theta).contiguous(),
                    torch.sin(phi).contiguous(), torch.cos(phi).contiguous(), grid_lin, hscale,
                    r, att, theta, phi, nt, nphi, r.shape[0])


def build_geometry(walls, box, ns, start, end, c, deltaT, volume_y, preset="torch", mode="noocl"):
    """All tables for P wall points.  walls [P,3] device tensor; box [8,3]; start/end are the
    reference's bin indices (configs/default.py:17-18); volume_y = volume_position[1]."""
    device = walls.device
    walls = walls.float().contiguous()
    box = box.to(device).float()
    tmin, tmax, pmin, pmax = angle_ranges(walls, box)
    extra = float(volume_y) ** 2                 # x Y^2, nlos_helpers.py:226 / :275-276
    if preset == "cuda" and mode in ("noocl", "binint"):
        extra = extra * (c * deltaT)             # volume_renderer.cu:182 (x c dT in-kernel)
    r, att, _, _ = radial_tables(start, end, c, deltaT, preset, device)
    return geometry_from_ranges(walls, tmin, tmax, pmin, pmax, ns, ns, r, att, extra)


def relay_wall_grid(H, W, extent=1.0, device=None):
    """Cell-centred H x W relay-wall points on the plane y=0 over x,z in [-extent/2, extent/2]
    (SURVEY §8d synthetic geometry).  Row-major [H*W, 3] with index m*W + n (nlos_helpers.py:303)."""
    zs = (torch.arange(H, dtype=torch.float64) + 0.5) / H * extent - extent / 2
    xs = (torch.arange(W, dtype=torch.float64) + 0.5) / W * extent - extent / 2
    zz, xx = torch.meshgrid(zs, xs, indexing="ij")
    pts = torch.stack([xx.reshape(-1), torch.zeros(H * W, dtype=torch.float64), zz.reshape(-1)], dim=1)
    return pts.float().to(device)
