"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py) — torch-CPU restatement of the reference.

Every function cites the reference file:line it restates (paths under /root/reference).
Two convention presets exist because the reference's three implementations disagree
(SURVEY.md Appendix A.3):

  preset "torch"  = path T, the default training path and the parity contract
                    (gaussian_model/gaussian_model.py:253-364, nlos_helpers.py:124-232)
  preset "cuda"   = path C, submodules/cuda_renderer/src/volume_renderer.cu:16-185 with
                    include/cuda_utils.cuh:54-151 and include/spherical_harmonics.cuh:20-80,
                    post-processing of gaussian_model/cuda_autograd.py:301-314

Gradients are torch autograd through these restatements (the reference's own backward for
path T is torch autograd too; path C's backward returns zeros, cuda_autograd.py:147-156).

An optional Mahalanobis cutoff `mc` zeroes every sample whose whitened squared distance
exceeds mc**2 — the exact support rule the HIP kernels implement; mc=None is the dense
reference semantics.
"""
import math

import torch

C0 = 0.28209479177387814
C1 = 0.4886025119029199
C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792,
      0.5462742152960396]
C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
      -0.4570457994644658, 1.445305721320277, -0.5900435899266435]
C4 = [2.5033429417967046, -1.7701307697799304, 0.9461746957575601, -0.6690465435572892,
      0.10578554691520431, -0.6690465435572892, 0.47308734787878004, -1.7701307697799304,
      0.6258357354491761]   # sh_utils.py:44-54


# --------------------------------------------------------------------------------------------
# geometry: nlos_helpers.py:87-188
# --------------------------------------------------------------------------------------------
def cartesian2spherical(pt):
    """nlos_helpers.py:87-95 — (x,y,z) -> (r, theta=acos(z/r), phi=atan2(y,x))."""
    out = torch.zeros(pt.shape, dtype=pt.dtype)
    r = torch.linalg.norm(pt, dim=1)
    out[:, 0] = r
    out[:, 1] = torch.acos(pt[:, 2] / r)
    out[:, 2] = torch.atan2(pt[:, 1], pt[:, 0])
    return out


def spherical2cartesian(pt):
    """nlos_helpers.py:98-104."""
    out = torch.zeros(pt.shape, dtype=pt.dtype)
    out[:, 0] = pt[:, 0] * torch.sin(pt[:, 1]) * torch.cos(pt[:, 2])
    out[:, 1] = pt[:, 0] * torch.sin(pt[:, 1]) * torch.sin(pt[:, 2])
    out[:, 2] = pt[:, 0] * torch.cos(pt[:, 1])
    return out


def volume_box_point(volume_position, volume_size):
    """nlos_helpers.py:107-118 — the 8 corners in the reference's order."""
    xv, yv, zv = [float(v) for v in volume_position]
    h = volume_size / 2
    x = [xv - h] * 4 + [xv + h] * 4
    y = [yv - h, yv - h, yv + h, yv + h] * 2
    z = [zv - h, zv + h] * 4
    return torch.tensor([x, y, z], dtype=torch.float64).t().float()


def sample_tables(p, box, ns, start, end, c, deltaT):
    """nlos_helpers.py:124-188 (spherical_sample_histogram) for ONE wall point p [3].

    Returns a dict with theta[ns], phi[ns], r[nr], I1, I2, dtheta, dphi, angle range and
    input_points [Nr*ns*ns, 5] in the reference's (k, i, j) flatten order."""
    bp = box - p[None, :]
    sph = cartesian2spherical(bp)
    tmin = torch.min(sph[:, 1]).item()
    tmax = torch.max(sph[:, 1]).item()
    pmin = torch.min(sph[:, 2]).item()
    pmax = torch.max(sph[:, 2]).item()
    theta = torch.linspace(tmin, tmax, ns, dtype=torch.float)
    phi = torch.linspace(pmin, pmax, ns, dtype=torch.float)
    dtheta = (tmax - tmin) / ns
    dphi = (pmax - pmin) / ns
    r_min = start * c * deltaT
    r_max = end * c * deltaT
    nr = end - start
    r = torch.linspace(r_min, r_max, nr, dtype=torch.float)
    I1 = math.floor(r_min / (c * deltaT))
    I2 = math.ceil(r_max / (c * deltaT))
    grid = torch.stack(torch.meshgrid(r, theta, phi, indexing="ij"), dim=-1)
    sph = grid.reshape(-1, 3)
    cart = spherical2cartesian(sph) + p
    ip = torch.cat((cart, sph[:, 1:3]), dim=1).float()
    return dict(theta=theta, phi=phi, r=r, I1=I1, I2=I2, nr=nr, dtheta=dtheta, dphi=dphi,
                theta_min=tmin, theta_max=tmax, phi_min=pmin, phi_max=pmax, input_points=ip)


# --------------------------------------------------------------------------------------------
# Gaussian math
# --------------------------------------------------------------------------------------------
def build_rotation(r):
    """gaussian_utils.py:189-210 — normalises (no eps) then the row-major rotation."""
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], dim=1)
    return R.reshape(-1, 3, 3)


def quat_to_rotmat_cuda(q):
    """cuda_utils.cuh:54-85 — identity when |q| < 1e-8, else normalise once."""
    norm = torch.sqrt((q * q).sum(dim=1))
    safe = torch.where(norm < 1e-8, torch.ones_like(norm), norm)
    qn = q / safe[:, None]
    R = build_rotation(qn)  # build_rotation re-normalises; |qn| == 1 up to rounding
    eye = torch.eye(3, dtype=q.dtype).expand_as(R)
    return torch.where((norm < 1e-8)[:, None, None], eye, R)


def eval_sh(deg, sh, dirs):
    """sh_utils.py:57-112 (3DGS sign convention), degrees 0..4."""
    assert 0 <= deg <= 4
    result = C0 * sh[..., 0]
    if deg > 0:
        x, y, z = dirs[..., 0:1], dirs[..., 1:2], dirs[..., 2:3]
        result = result - C1 * y * sh[..., 1] + C1 * z * sh[..., 2] - C1 * x * sh[..., 3]
        if deg > 1:
            xx, yy, zz = x * x, y * y, z * z
            xy, yz, xz = x * y, y * z, x * z
            result = (result + C2[0] * xy * sh[..., 4] + C2[1] * yz * sh[..., 5]
                      + C2[2] * (2.0 * zz - xx - yy) * sh[..., 6]
                      + C2[3] * xz * sh[..., 7] + C2[4] * (xx - yy) * sh[..., 8])
            if deg > 2:
                result = (result + C3[0] * y * (3 * xx - yy) * sh[..., 9]
                          + C3[1] * xy * z * sh[..., 10]
                          + C3[2] * y * (4 * zz - xx - yy) * sh[..., 11]
                          + C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[..., 12]
                          + C3[4] * x * (4 * zz - xx - yy) * sh[..., 13]
                          + C3[5] * z * (xx - yy) * sh[..., 14]
                          + C3[6] * x * (xx - 3 * yy) * sh[..., 15])
                if deg > 3:   # sh_utils.py:102-112
                    result = (result + C4[0] * xy * (xx - yy) * sh[..., 16]
                              + C4[1] * yz * (3 * xx - yy) * sh[..., 17]
                              + C4[2] * xy * (7 * zz - 1) * sh[..., 18]
                              + C4[3] * yz * (7 * zz - 3) * sh[..., 19]
                              + C4[4] * (zz * (35 * zz - 30) + 3) * sh[..., 20]
                              + C4[5] * xz * (7 * zz - 3) * sh[..., 21]
                              + C4[6] * (xx - yy) * (7 * zz - 1) * sh[..., 22]
                              + C4[7] * xz * (xx - 3 * yy) * sh[..., 23]
                              + C4[8] * (xx * (xx - 3 * yy) - yy * (3 * xx - yy)) * sh[..., 24])
    return result


def eval_sh_cuda(deg, sh, dirs):
    """spherical_harmonics.cuh:20-80 — same basis WITHOUT the 3DGS sign flips, and the
    (3z^2-1), (5z^2-1), (5z^2-3) polynomial forms.  sh: [..., K], dirs: [..., 3] -> [...]."""
    x, y, z = dirs[..., 0], dirs[..., 1], dirs[..., 2]
    basis = [torch.full_like(x, C0)]
    if deg >= 1:
        basis += [C1 * y, C1 * z, C1 * x]
    if deg >= 2:
        basis += [1.0925484305920792 * x * y, 1.0925484305920792 * y * z,
                  0.31539156525252005 * (3.0 * z * z - 1.0), 1.0925484305920792 * x * z,
                  0.5462742152960396 * (x * x - y * y)]
    if deg >= 3:
        basis += [0.5900435899266435 * y * (3.0 * x * x - y * y), 2.890611442640554 * x * y * z,
                  0.4570457994644658 * y * (5.0 * z * z - 1.0),
                  0.3731763325901154 * z * (5.0 * z * z - 3.0),
                  0.4570457994644658 * x * (5.0 * z * z - 1.0),
                  1.445305721320277 * z * (x * x - y * y),
                  0.5900435899266435 * x * (x * x - 3.0 * y * y)]
    out = torch.zeros_like(x)
    for i, b in enumerate(basis):
        out = out + sh[..., i] * b
    return out


class Params:
    """Raw Gaussian parameters with the reference GaussianModel's names
    (gaussian_model/gaussian_model.py:38-49, features layout :120-123, :195-218)."""

    def __init__(self, mu, scaling, rotation, opacity, features_dc, features_rest, active_sh_degree,
                 requires_grad=True):
        t = lambda a: torch.as_tensor(a, dtype=torch.float32).clone().requires_grad_(requires_grad)
        self._mu = t(mu)
        self._scaling = t(scaling)
        self._rotation = t(rotation)
        self._opacity = t(opacity)
        self._features_dc = t(features_dc)
        self._features_rest = t(features_rest)
        self.active_sh_degree = int(active_sh_degree)

    @property
    def features(self):
        return torch.cat((self._features_dc, self._features_rest), dim=1)  # [Ng, K, 1]

    def leaves(self):
        return [self._mu, self._scaling, self._rotation, self._opacity, self._features_dc,
                self._features_rest]


def gaussian_pdf(x, P, preset="torch", mod=1.0, mc=None):
    """pdf [Ng, Na].

    torch: gaussian_model.py:253-294  s = exp(exp(_scaling)*mod), u = R(q̂)(x-μ), no eps.
    cuda : cuda_utils.cuh:124-151     s = exp(_scaling)*mod,    u = Rᵀ(x-μ), /(s+1e-8)."""
    if preset == "torch":
        scales = torch.exp(torch.exp(P._scaling) * mod)
        rots = build_rotation(torch.nn.functional.normalize(P._rotation))
        diff = x.unsqueeze(0) - P._mu.unsqueeze(1)
        T = torch.matmul(rots.unsqueeze(1), diff.unsqueeze(-1)).squeeze(-1)
        m2 = torch.sum((T / scales.unsqueeze(1)) ** 2, dim=-1)
    else:
        scales = torch.exp(P._scaling) * mod + 1e-8
        rots = quat_to_rotmat_cuda(P._rotation)
        diff = x.unsqueeze(0) - P._mu.unsqueeze(1)
        T = torch.matmul(rots.transpose(1, 2).unsqueeze(1), diff.unsqueeze(-1)).squeeze(-1)
        m2 = torch.sum((T / scales.unsqueeze(1)) ** 2, dim=-1)
    pdf = torch.exp(-0.5 * m2)
    if mc is not None:
        pdf = torch.where(m2 <= mc * mc, pdf, torch.zeros_like(pdf))
    return pdf


def albedo(P, p, preset="torch", deg=None):
    """ρ_g(p) = max(0, 0.5 + SH(d̂)·f), d̂ = (μ-p)/|μ-p|.
    torch: gaussian_model.py:350-355 (eval_sh, /norm, no eps); cuda: volume_renderer.cu:109-111."""
    deg = P.active_sh_degree if deg is None else deg
    d = P._mu - p.unsqueeze(0)
    if preset == "torch":
        dn = d / d.norm(dim=1, keepdim=True)
        K = P.features.shape[1]
        shs = P.features.transpose(1, 2).view(-1, 1, K)
        sh = eval_sh(deg, shs, dn)  # [Ng, 1]
    else:
        dn = d * (1.0 / (torch.sqrt((d * d).sum(dim=1, keepdim=True)) + 1e-8))
        f = P.features[:, :, 0]
        sh = eval_sh_cuda(deg, f, dn).unsqueeze(1)
    return torch.clamp_min(sh + 0.5, 0.0)  # [Ng, 1]


# --------------------------------------------------------------------------------------------
# one wall point: gaussian_transient_rendering (nlos_helpers.py:192-232)
# --------------------------------------------------------------------------------------------
def render_wallpoint(P, p, tab, Y, c, deltaT, preset="torch", mode="noocl", mod=1.0, mc=None):
    """Returns (result [Nr, Ns*Ns], hist [Nr]).

    torch preset, mode 'noocl' : gaussian_model.py:346-364 + nlos_helpers.py:206-232
    torch preset, mode 'netf'  : gaussian_model.py:297-325 (per-Gaussian self-transmittance)
    cuda preset,  mode 'noocl' : volume_renderer.cu:138-183 (×cΔT) + cuda_autograd.py:301-314
                                 (/(t²+1e-8)·sinθ, Σ·dθdφ) + nlos_helpers.py:275-276 (×Y²)."""
    ns = tab["theta"].shape[0]
    nr = tab["r"].shape[0]
    x = tab["input_points"][:, 0:3]
    pdf = gaussian_pdf(x, P, preset, mod, mc)
    sig = torch.sigmoid(P._opacity)
    rho = albedo(P, p, preset)
    if mode == "noocl":
        rho_density = torch.sum(pdf * sig * rho, dim=0)
        if preset == "cuda":
            rho_density = rho_density * c * deltaT
    elif mode == "netf":
        density = (pdf * sig).view(-1, nr, ns * ns)
        occl = torch.exp(-density * c * deltaT)
        trans = torch.cumprod(torch.cat([torch.ones([occl.shape[0], 1, occl.shape[2]]), occl + 1e-7], 1),
                              1)[:, :-1, :]
        rho_density = torch.sum(density.view(-1, nr * ns * ns) * trans.view(-1, nr * ns * ns) * rho,
                                dim=0) * c * deltaT
    else:
        raise ValueError(mode)
    result = rho_density.reshape(nr, ns * ns)
    theta_grid = tab["input_points"].view(-1, ns * ns, 5)[:, :, 3]
    if preset == "torch":
        dist = (torch.linspace(tab["I1"], tab["I2"], nr, dtype=torch.float) * deltaT * c).view(-1, 1)
        result = result / (dist ** 2) * torch.sin(theta_grid)
    else:
        t = torch.linspace(tab["I1"] * c * deltaT, tab["I2"] * c * deltaT, nr).view(-1, 1)
        result = result / (t ** 2 + 1e-8) * torch.sin(theta_grid)
    result = result * (Y ** 2)
    hist = torch.sum(result, dim=1) * tab["dtheta"] * tab["dphi"]
    return result, hist


def render_volume(P, walls, box, Y, ns, start, end, c, deltaT, **kw):
    """Loop of render_wallpoint over wall points [P,3] -> hist [P, Nr] (the reference renders one
    wall point per step, main.py:198-269; the volume is the stack of those histograms)."""
    hs = []
    for w in range(walls.shape[0]):
        tab = sample_tables(walls[w], box, ns, start, end, c, deltaT)
        _, h = render_wallpoint(P, walls[w], tab, Y, c, deltaT, **kw)
        hs.append(h)
    return torch.stack(hs)


def count_support(P, walls, box, ns, start, end, c, deltaT, preset="cuda", mc=3.0, mod=1.0):
    """Number of in-support evaluations (wall point, Gaussian, ray, bin) with Mahalanobis² ≤ mc²
    and albedo > 0 — the work unit of SURVEY §8d (not a reference function; it counts the
    nonzero terms of the gaussian_pdf × albedo product the reference sums)."""
    n = 0
    for w in range(walls.shape[0]):
        tab = sample_tables(walls[w], box, ns, start, end, c, deltaT)
        pdf = gaussian_pdf(tab["input_points"][:, 0:3], P, preset, mod, mc)
        live = (albedo(P, walls[w], preset) > 0).float()
        n += int(((pdf > 0).float() * live).sum())
    return n


def mse_loss(hist, target):
    """compute_loss: MSELoss(mean) vs target (already × gt_times), nlos_helpers.py:323-327."""
    loss = torch.mean((hist - target) ** 2)
    return loss, loss / torch.mean(target ** 2)


# --------------------------------------------------------------------------------------------
# path C "rays" API: _C.filter_gaussians_per_ray + _C.render_rays (volume_renderer.cu:16-305)
# --------------------------------------------------------------------------------------------
def bboxes_cuda(P, mod=1.0, sigma=3.0):
    """bbox_compute.cuh:23-120 — [Ng, 6] (min xyz, max xyz); extent_i = sigma |R_i . s|, s = exp(S) mod
    (no +1e-8 here), R from quat_to_rotmat (cuda_utils.cuh:54-85)."""
    s = torch.exp(P._scaling) * mod
    R = quat_to_rotmat_cuda(P._rotation)
    ext = sigma * torch.sqrt(((R * s[:, None, :]) ** 2).sum(-1))
    return torch.cat([P._mu - ext, P._mu + ext], dim=1)


def bboxes_torch(P, mod=1.0, sigma=3.0):
    """gaussian_model.py:140-178 GaussianModel.get_bboxes — [Ng, 6]: L = build_rotation(normalize(q)) @
    diag(exp(S) mod) (gaussian_utils.py:212-221), extent = sigma sqrt(clamp_min(diag(L Lᵀ), 1e-8))."""
    s = torch.exp(P._scaling) * mod
    R = build_rotation(torch.nn.functional.normalize(P._rotation))
    L = R * s[:, None, :]
    cov = L @ L.transpose(1, 2)
    ext = sigma * torch.sqrt(torch.clamp_min(torch.diagonal(cov, dim1=-2, dim2=-1), 1e-8))
    return torch.cat([P._mu - ext, P._mu + ext], dim=1)


def aabb_filter(ray_o, ray_d, bboxes, cap=256):
    """ray_aabb.cu:10-61 + cuda_utils.cuh:97-121 — int32 [N_rays, cap+1]: count, then the first
    `cap` Gaussian indices (index order) whose box the half-infinite ray hits, -1 padding."""
    inv = 1.0 / (ray_d + 1e-8)                                        # [R,3]
    t0 = (bboxes[None, :, 0:3] - ray_o[:, None, :]) * inv[:, None, :]  # [R,Ng,3]
    t1 = (bboxes[None, :, 3:6] - ray_o[:, None, :]) * inv[:, None, :]
    tmin = torch.minimum(t0, t1).amax(-1)
    tmax = torch.maximum(t0, t1).amin(-1)
    hit = (tmax >= tmin) & (tmax >= 0)
    out = torch.full((ray_o.shape[0], cap + 1), -1, dtype=torch.int32)
    for r in range(ray_o.shape[0]):
        idx = torch.nonzero(hit[r]).flatten()[:cap]
        out[r, 0] = idx.numel()
        out[r, 1:1 + idx.numel()] = idx.to(torch.int32)
    return out


def render_rays_cuda(ray_o, ray_d, t, P, sh_features, cam, deg, c, deltaT, mod, use_occlusion, filt=None,
                     mc=None):
    """Per-(ray, sample) outputs (rho_density, density, transmittance) [N_rays, N_samples].

    volume_renderer.cu:16-185: each ray sums over the Gaussians of its filter row (all when
    filt is None).  No occlusion (:138-183): rho = cΔT Σ σ pdf ρ, T = 1.  Occlusion (:80-137):
    shared T across Gaussians, T_{s+1} = T_s exp(-D_s cΔT), rho = T Σ (1 - exp(-σ pdf cΔT)) ρ, and
    after the first step with T_{s+1} < 1e-4 all three outputs are zero (early exit), i.e. a
    sample is live iff T_s >= 1e-4."""
    nrays, nsamp = ray_o.shape[0], t.shape[0]
    x = (ray_o[:, None, :] + ray_d[:, None, :] * t[None, :, None]).reshape(-1, 3)
    pdf = gaussian_pdf(x, P, "cuda", mod, mc).view(-1, nrays, nsamp)   # [Ng, R, S]
    if filt is not None:
        mask = torch.zeros(P._mu.shape[0], nrays)
        for r in range(nrays):
            n = int(filt[r, 0])
            if n > 0:
                mask[filt[r, 1:1 + n].long(), r] = 1.0
        pdf = pdf * mask[:, :, None]
    sig = torch.sigmoid(P._opacity).view(-1, 1, 1)
    d = P._mu - cam.unsqueeze(0)
    dn = d * (1.0 / (torch.sqrt((d * d).sum(dim=1, keepdim=True)) + 1e-8))
    rho = torch.clamp_min(eval_sh_cuda(deg, sh_features, dn) + 0.5, 0.0).view(-1, 1, 1)
    contrib = pdf * sig
    density = contrib.sum(0)
    if not use_occlusion:
        rho_density = (contrib * rho).sum(0) * c * deltaT
        return rho_density, density, torch.ones_like(density)
    wa = ((1.0 - torch.exp(-contrib * c * deltaT)) * rho).sum(0)
    step = torch.exp(-density * c * deltaT)
    T = torch.cumprod(torch.cat([torch.ones(nrays, 1), step[:, :-1]], dim=1), dim=1)
    live = (T >= 1e-4).float()
    return T * wa * live, density * live, T * live



# --------------------------------------------------------------------------------------------
# C4 "analytic_exact": per-bin exact integral of the numerical model (not a reference function;
# SURVEY §8d C4 — the corrected counterpart of the analytic section path, cross-checked against
# the point-sampled numerical path at the same support)
# --------------------------------------------------------------------------------------------
def _erf_diff(x0, x1):
    """erf(x1) - erf(x0) for x0 <= x1 without tail cancellation (erfc on the far side)."""
    e0, e1 = torch.special.erfc(x0.abs()), torch.special.erfc(x1.abs())
    return torch.where(x0 >= 0, e0 - e1, torch.where(x1 <= 0, e1 - e0, 2.0 - e0 - e1))


def bin_integrated_pdf(P, p, tab, preset="cuda", mod=1.0, mc=None):
    """[Ng, Na] in the (k, i, j) order of input_points: the average of pdf_g over the radial bin
    [r_k - dr/2, r_k + dr/2] of ray (i, j), in float64.  Along a ray u(r) = u0 + r v, so
    pdf = exp(-m2min/2) exp(-a (r - t*)^2 / 2) and the bin average is
    exp(-m2min/2) sqrt(pi)/(2 beta) [erf(beta (kap + 1/2)) - erf(beta (kap - 1/2))],
    beta = dr sqrt(a/2), kap = (r_k - t*)/dr.  The support mask is the numerical path's
    (m^2 at the bin centre <= mc^2, gaussian_pdf)."""
    f64 = torch.float64
    theta, phi, r = tab["theta"].to(f64), tab["phi"].to(f64), tab["r"].to(f64)
    ns, nr = theta.shape[0], r.shape[0]
    dirs = torch.stack([torch.sin(theta)[:, None] * torch.cos(phi)[None, :],
                        torch.sin(theta)[:, None] * torch.sin(phi)[None, :],
                        torch.cos(theta)[:, None].expand(ns, ns)], dim=-1).reshape(-1, 3)   # [ns*ns, 3]
    if preset == "torch":
        s = torch.exp(torch.exp(P._scaling) * mod).to(f64)
        Rot = build_rotation(torch.nn.functional.normalize(P._rotation)).to(f64)
    else:
        s = (torch.exp(P._scaling) * mod + 1e-8).to(f64)
        Rot = quat_to_rotmat_cuda(P._rotation).transpose(1, 2).to(f64)
    mu = P._mu.to(f64)
    u0 = torch.einsum("gab,gb->ga", Rot, p.to(f64)[None, :] - mu) / s                 # [Ng, 3]
    v = torch.einsum("gab,nb->gna", Rot, dirs) / s[:, None, :]                         # [Ng, R, 3]
    a = (v * v).sum(-1)
    ts = -(u0[:, None, :] * v).sum(-1) / a
    zs = u0[:, None, :] + ts[..., None] * v
    m2min = (zs * zs).sum(-1)
    dr = (r[-1] - r[0]) / (nr - 1)
    beta = dr * torch.sqrt(a / 2)                                                      # [Ng, R]
    kap = (r[None, :, None] - ts[:, None, :]) / dr                                     # [Ng, nr, R]
    diff = _erf_diff(beta[:, None, :] * (kap - 0.5), beta[:, None, :] * (kap + 0.5))
    val = torch.exp(-0.5 * m2min)[:, None, :] * math.sqrt(math.pi) / (2 * beta[:, None, :]) * diff
    val = val.reshape(P._mu.shape[0], -1)
    if mc is not None:
        live = gaussian_pdf(tab["input_points"][:, 0:3], P, preset, mod, mc) > 0
        val = torch.where(live, val, torch.zeros_like(val))
    return val


def render_volume_binint(P, walls, box, Y, ns, start, end, c, deltaT, preset="cuda", mod=1.0, mc=None):
    """hist [P, Nr] of the no-occlusion path with bin_integrated_pdf in place of the point pdf
    (attenuation, sin(theta), angular sum and scales exactly as render_wallpoint)."""
    hs = []
    for w in range(walls.shape[0]):
        p = walls[w]
        tab = sample_tables(p, box, ns, start, end, c, deltaT)
        nr = tab["r"].shape[0]
        pdf = bin_integrated_pdf(P, p, tab, preset, mod, mc)
        sig = torch.sigmoid(P._opacity).to(torch.float64)
        rho = albedo(P, p, preset).to(torch.float64)
        rd = torch.sum(pdf * sig * rho, dim=0)
        if preset == "cuda":
            rd = rd * c * deltaT
        result = rd.reshape(nr, ns * ns)
        theta_grid = tab["input_points"].view(-1, ns * ns, 5)[:, :, 3].to(torch.float64)
        if preset == "torch":
            dist = (torch.linspace(tab["I1"], tab["I2"], nr, dtype=torch.float) * deltaT * c).view(-1, 1)
            result = result / (dist.to(torch.float64) ** 2) * torch.sin(theta_grid)
        else:
            t = torch.linspace(tab["I1"] * c * deltaT, tab["I2"] * c * deltaT, nr).view(-1, 1)
            result = result / (t.to(torch.float64) ** 2 + 1e-8) * torch.sin(theta_grid)
        hs.append(torch.sum(result * Y ** 2, dim=1) * tab["dtheta"] * tab["dphi"])
    return torch.stack(hs)


# --------------------------------------------------------------------------------------------
# path A: the analytic section renderer (_C.render_rays_analytic)
# --------------------------------------------------------------------------------------------
def render_rays_analytic(ray_o, ray_d, t_min, t_max, filt, P, sh_features, cam, deg, mod=1.0, sigma=3.0):
    """One value per ray, volume_renderer_analytic.cu:23-173 with analytic_integration.cuh:38-192.

    Per ray: the first 128 filter entries (in filter order) whose sigma-ellipsoid the line hits
    (compute_gaussian_section :38-104; s = exp(S) mod with no eps, local = R^T (x - mu)), entry/exit
    clipped to [t_min, t_max] and kept iff t_enter < t_exit; stable sort by t_enter (insertion sort
    :178-192); per section tau = max(0, G e^{-(a - b^2/4c)/2} [erf((b + 2c t1)/(2 sqrt c)) -
    erf((b + 2c t0)/(2 sqrt c))]), G = sigma_o sqrt(2 pi / c) sx sy sz (:123-172, the reference's
    formula as written); acc += T (1 - e^-tau) rho, T *= e^-tau, stop once T < 1e-4 (:118-170).
    rho = max(0, 0.5 + SH_cuda(deg, f_g, normalize_eps(mu - cam))) (:148-151).  Pure-Python loop
    over rays: small cases only."""
    ng = P._mu.shape[0]
    out = torch.zeros(ray_o.shape[0])
    s_all = torch.exp(P._scaling) * mod
    R_all = quat_to_rotmat_cuda(P._rotation)
    sig_all = torch.sigmoid(P._opacity).reshape(-1)
    d = P._mu - cam[None, :]
    dn = d * (1.0 / (torch.sqrt((d * d).sum(dim=1, keepdim=True)) + 1e-8))
    rho_all = torch.clamp_min(eval_sh_cuda(deg, sh_features, dn) + 0.5, 0.0)
    for ray in range(ray_o.shape[0]):
        o, dv = ray_o[ray], ray_d[ray]
        n = int(filt[ray, 0])
        secs = []
        for e in range(n):
            if len(secs) >= 128:
                break
            g = int(filt[ray, 1 + e])
            if g < 0 or g >= ng:
                continue
            Rt = R_all[g].t()
            so = (Rt @ (o - P._mu[g])) / s_all[g]
            sd = (Rt @ dv) / s_all[g]
            a = torch.dot(sd, sd)
            b = 2.0 * torch.dot(so, sd)
            cc = torch.dot(so, so) - sigma * sigma
            disc = b * b - 4.0 * a * cc
            if disc < 0:
                continue
            sq = torch.sqrt(disc)
            te = torch.clamp_min((-b - sq) / (2.0 * a), t_min)
            tx = torch.clamp_max((-b + sq) / (2.0 * a), t_max)
            if te < tx:
                secs.append((g, float(te), float(tx), so, sd))
        secs.sort(key=lambda x: x[1])   # stable, as the insertion sort
        T, acc = 1.0, 0.0
        for g, te, tx, so, sd in secs:
            A = torch.dot(so, so)
            B = 2.0 * torch.dot(so, sd)
            C = torch.dot(sd, sd)
            G = sig_all[g] * torch.sqrt(2.0 * math.pi / C) * s_all[g].prod()
            ef = torch.exp(-0.5 * (A - B * B / (4.0 * C)))
            e1 = torch.special.erf((B + 2.0 * C * tx) / (2.0 * torch.sqrt(C)))
            e0 = torch.special.erf((B + 2.0 * C * te) / (2.0 * torch.sqrt(C)))
            tau = torch.clamp_min(G * ef * (e1 - e0), 0.0)
            st = torch.exp(-tau)
            acc = acc + T * (1.0 - st) * rho_all[g]
            T = T * st
            if T < 1e-4:
                break
        out[ray] = acc
    return out


def render_rays_analytic_batched(ray_o, ray_d, t_min, t_max, filt, P, sh_features, cam, deg, mod=1.0, sigma=3.0,
                                 chunk=2048, dtype=None):
    """render_rays_analytic (above, the line-by-line restatement of volume_renderer_analytic.cu:23-173)
    vectorised over rays and filter entries, for the C4-size cross-check of path A (test
    infrastructure; pinned to the loop version by tests/test_oracle_analytic_cpu.py).  Same rules:
    the first 128 filter entries (filter order) whose sigma-ellipsoid section is non-empty after the
    [t_min, t_max] clip, stable sort by t_enter, tau clamped >= 0, front-to-back compositing that
    stops once T < 1e-4 (a section contributes iff the transmittance before it is >= 1e-4).
    dtype=torch.float64 evaluates the same formula in double precision: with small Gaussians tau is
    ~1e-7 and the reference's fp32 1 - exp(-tau) is all cancellation, so parity is judged against
    the formula's exact value (the HIP kernel evaluates 1 - exp(-tau) as -expm1(-tau))."""
    if dtype is not None:
        from types import SimpleNamespace
        cv = lambda t: t.to(dtype)
        P = SimpleNamespace(_mu=cv(P._mu), _scaling=cv(P._scaling), _rotation=cv(P._rotation),
                            _opacity=cv(P._opacity))
        ray_o, ray_d, sh_features, cam = cv(ray_o), cv(ray_d), cv(sh_features), cv(cam)
    ng = P._mu.shape[0]
    s_all = torch.exp(P._scaling) * mod
    R_all = quat_to_rotmat_cuda(P._rotation)
    sig_all = torch.sigmoid(P._opacity).reshape(-1)
    d = P._mu - cam[None, :]
    dn = d * (1.0 / (torch.sqrt((d * d).sum(dim=1, keepdim=True)) + 1e-8))
    rho_all = torch.clamp_min(eval_sh_cuda(deg, sh_features, dn) + 0.5, 0.0).reshape(-1)
    out = torch.zeros(ray_o.shape[0], dtype=ray_o.dtype)
    ne = filt.shape[1] - 1
    for r0 in range(0, ray_o.shape[0], chunk):
        o = ray_o[r0:r0 + chunk]
        dv = ray_d[r0:r0 + chunk]
        f = filt[r0:r0 + chunk]
        n = f[:, 0:1].long()
        gi = f[:, 1:].long()
        ent = torch.arange(ne).view(1, -1)
        ok = (ent < n) & (gi >= 0) & (gi < ng)
        g = torch.where(ok, gi, torch.zeros_like(gi))
        Rt = R_all[g].transpose(-1, -2)                                    # [n, ne, 3, 3]
        so = (Rt @ (o[:, None, :] - P._mu[g]).unsqueeze(-1)).squeeze(-1) / s_all[g]
        sd = (Rt @ dv[:, None, :].expand(-1, ne, -1).unsqueeze(-1)).squeeze(-1) / s_all[g]
        a = (sd * sd).sum(-1)
        b = 2.0 * (so * sd).sum(-1)
        cc = (so * so).sum(-1) - sigma * sigma
        disc = b * b - 4.0 * a * cc
        sq = torch.sqrt(torch.clamp_min(disc, 0.0))
        te = torch.clamp_min((-b - sq) / (2.0 * a), t_min)
        tx = torch.clamp_max((-b + sq) / (2.0 * a), t_max)
        sec = ok & (disc >= 0) & (te < tx)
        sec = sec & (torch.cumsum(sec.long(), dim=1) <= 128)               # the 128-section cap
        key = torch.where(sec, te, torch.full_like(te, float("inf")))
        order = torch.sort(key, dim=1, stable=True).indices
        take = lambda t: torch.gather(t, 1, order)
        sec_s = take(sec)
        A = take((so * so).sum(-1))
        B = take(b)
        C = take(a)
        gs = take(g)
        te_s, tx_s = take(te), take(tx)
        G = sig_all[gs] * torch.sqrt(2.0 * math.pi / C) * s_all[gs].prod(-1)
        ef = torch.exp(-0.5 * (A - B * B / (4.0 * C)))
        e1 = torch.special.erf((B + 2.0 * C * tx_s) / (2.0 * torch.sqrt(C)))
        e0 = torch.special.erf((B + 2.0 * C * te_s) / (2.0 * torch.sqrt(C)))
        tau = torch.where(sec_s, torch.clamp_min(G * ef * (e1 - e0), 0.0), torch.zeros_like(A))
        st = torch.exp(-tau)
        T_incl = torch.cumprod(st, dim=1)
        T_excl = torch.cat([torch.ones_like(T_incl[:, :1]), T_incl[:, :-1]], dim=1)
        live = sec_s & (T_excl >= 1e-4)
        contrib = torch.where(live, T_excl * (1.0 - st) * rho_all[gs], torch.zeros_like(A))
        out[r0:r0 + chunk] = torch.cumsum(contrib, dim=1)[:, -1]
    return out
