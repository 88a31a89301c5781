"""Drop-in counterparts of the reference's nlos_helpers.py hot-path functions, rendered by the
HIP kernels (no dense [Ng, Na] torch tensors).

    CUDA_AVAILABLE, CUDA_RENDERER          nlos_helpers.py:21-27       (created at import; None without a GPU)
    spherical_sample_histogram             nlos_helpers.py:124-188     (same return tuple)
    gaussian_transient_rendering           nlos_helpers.py:192-232     (same signature and outputs, real grads;
                                                                        args.use_cuda_renderer dispatch :200-204)
    gaussian_transient_rendering_cuda      nlos_helpers.py:235-278     (path C through GaussianRendererCUDA,
                                                                        x Y^2 on both outputs)
    compute_loss                           nlos_helpers.py:280-346     (same loss / equal_loss; no per-step .mat
                                                                        dump unless args.save_loss_mat is set)
Without args.use_cuda_renderer the default path T conventions apply (preset "torch"); args.occlusion
selects the 'netf' self-transmittance model like gaussian_model.py:297-325.  args.render_cutoff
(optional, default 0 = dense, the reference's exact semantics) enables support culling at that
Mahalanobis radius.  With args.use_cuda_renderer set and a GPU present, rendering goes through path C
(volume_renderer.cu conventions, shared transmittance when args.occlusion) exactly as the reference
dispatches it; without a GPU the reference falls back to path T, and so does this module (whose
path T then raises, since there is no CPU renderer).
"""
import math

import torch

from .geometry import geometry_from_ranges
from .model import features_flat
from .render import RenderConfig, render
from .rendering_cuda import CUDA_AVAILABLE, create_cuda_renderer  # noqa: F401

# nlos_helpers.py:21-27: the path-C renderer is created at import time (None when unavailable)
CUDA_RENDERER = create_cuda_renderer()


def cartesian2spherical_torch(pt):
    """nlos_helpers.py:87-95."""
    out = torch.zeros(pt.shape, device=pt.device)
    r = torch.linalg.norm(pt, dim=1)
    out[:, 0] = r
    out[:, 1] = torch.acos(pt[:, 2] / r)
    out[:, 2] = torch.atan2(pt[:, 1], pt[:, 0])
    return out


def spherical2cartesian_torch(pt):
    """nlos_helpers.py:98-104."""
    out = torch.zeros(pt.shape, device=pt.device)
    out[:, 0] = pt[:, 0] * torch.sin(pt[:, 1]) * torch.cos(pt[:, 2])
    out[:, 1] = pt[:, 0] * torch.sin(pt[:, 1]) * torch.sin(pt[:, 2])
    out[:, 2] = pt[:, 0] * torch.cos(pt[:, 1])
    return out


def spherical_sample_histogram(args, data_kwargs, current_camera_grid_positions):
    """Same outputs as nlos_helpers.py:124-188: (input_points [Nr*Ns^2, 5], I1, I2, num_r, dtheta,
    dphi, theta_min, theta_max, phi_min, phi_max)."""
    assert isinstance(current_camera_grid_positions, torch.Tensor)
    box = data_kwargs["volume_box_point"]
    device = box.device
    sph = cartesian2spherical_torch(box - current_camera_grid_positions[None, :])
    theta_min = torch.min(sph[:, 1]).item()
    theta_max = torch.max(sph[:, 1]).item()
    phi_min = torch.min(sph[:, 2]).item()
    phi_max = torch.max(sph[:, 2]).item()
    ns = args.num_sampling_points
    theta = torch.linspace(theta_min, theta_max, ns, dtype=torch.float, device=device)
    phi = torch.linspace(phi_min, phi_max, ns, dtype=torch.float, device=device)
    dtheta = (theta_max - theta_min) / ns
    dphi = (phi_max - phi_min) / ns
    c, deltaT = data_kwargs["c"], data_kwargs["deltaT"]
    r_min = args.start * c * deltaT
    r_max = args.end * c * deltaT
    num_r = args.end - args.start
    r = torch.linspace(r_min, r_max, num_r, dtype=torch.float, device=device)
    I1 = math.floor(r_min / (c * deltaT))
    I2 = math.ceil(r_max / (c * deltaT))
    grid = torch.stack(torch.meshgrid(r, theta, phi, indexing="ij"), dim=-1)
    spherical = grid.reshape([-1, 3])
    cart = spherical2cartesian_torch(spherical) + current_camera_grid_positions
    cart = torch.cat((cart, spherical[:, 1:3]), dim=1).float()
    return cart, I1, I2, r.shape[0], dtheta, dphi, theta_min, theta_max, phi_min, phi_max


def _mode(args):
    if not args.occlusion:
        return "noocl"
    rt = str(getattr(args, "rendering_type", "netf")).lower()
    if rt == "netf":
        return "netf"
    # gaussian_model.py:326-339 raises a shape error for 'nlos-neus'; reject it explicitly
    raise NotImplementedError(f"rendering_type {rt!r} is not supported (the reference crashes on it)")


def gaussian_transient_rendering(args, model, data_kwargs, input_points, current_camera_grid_positions, I1, I2,
                                 num_r, dtheta, dphi):
    """(result [num_r, Ns^2], pred_histogram [num_r]) exactly as nlos_helpers.py:192-232 defines them,
    with the dense Gaussian evaluation replaced by the HIP renderer.  args.use_cuda_renderer routes to
    gaussian_transient_rendering_cuda when the path-C renderer exists (:200-204)."""
    if getattr(args, "use_cuda_renderer", False) and CUDA_RENDERER is not None:
        return gaussian_transient_rendering_cuda(args, model, data_kwargs, input_points, current_camera_grid_positions,
                                                 I1, I2, num_r, dtheta, dphi)
    ns = args.num_sampling_points
    dev = input_points.device
    c, deltaT = data_kwargs["c"], data_kwargs["deltaT"]
    ip = input_points.view(num_r, ns, ns, 5)
    theta = ip[0, :, 0, 3].reshape(1, ns).contiguous()
    phi = ip[0, 0, :, 4].reshape(1, ns).contiguous()
    cam = current_camera_grid_positions.reshape(1, 3).float()
    r = torch.linspace(args.start * c * deltaT, args.end * c * deltaT, num_r, dtype=torch.float, device=dev)
    with torch.no_grad():
        dist = torch.linspace(I1, I2, num_r, dtype=torch.float, device=dev) * deltaT * c
    att = (1.0 / dist ** 2).contiguous()
    Y = data_kwargs["volume_position"][1]
    Yf = float(Y)
    geo = geometry_from_ranges(cam, theta[:, 0], theta[:, -1], phi[:, 0], phi[:, -1], ns, ns, r, att,
                               hscale_extra=Yf * Yf, theta=theta, phi=phi)
    # exact dtheta/dphi passed by the caller (already (max-min)/Ns)
    geo.hscale = torch.tensor([dtheta * dphi * Yf * Yf], dtype=torch.float, device=dev)
    mode = _mode(args)
    cfg = RenderConfig(preset="torch", mode=mode, sh_degree=int(model.active_sh_degree),
                       scaling_modifier=float(args.scaling_modifier),
                       cutoff=float(getattr(args, "render_cutoff", 0.0) or 0.0), c_deltaT=float(c * deltaT))
    hist, rays = render(model._mu, model._scaling, model._rotation, model._opacity, features_flat(model), geo, cfg,
                        want_hist=True, want_rays=True)
    # post-processing in the reference's op order (nlos_helpers.py:216-226) on the per-ray rho_density
    result = rays[0].t().reshape(num_r, ns * ns)
    Theta = ip[:, :, :, 3].reshape(num_r, ns * ns)
    result = result / (dist.view(-1, 1) ** 2) * torch.sin(Theta)
    result = result * (Y ** 2)
    return result, hist[0]


def gaussian_transient_rendering_cuda(args, model, data_kwargs, input_points, current_camera_grid_positions, I1, I2,
                                      num_r, dtheta, dphi):
    """nlos_helpers.py:235-278: angular ranges recovered from input_points, r_range = (I1, I2) c dT,
    GaussianRendererCUDA.render_transient (path C: ray grid, per-ray box filter, volume_renderer.cu
    sampling, /(t^2 + 1e-8) sin(theta), angular sum), then x Y^2 on result and pred_histogram.
    dtheta / dphi are recomputed by the renderer from the ranges, as in the reference."""
    theta_vals = input_points[:, 3]
    phi_vals = input_points[:, 4]
    theta_min = theta_vals.min().item()
    theta_max = theta_vals.max().item()
    phi_min = phi_vals.min().item()
    phi_max = phi_vals.max().item()
    c, deltaT = data_kwargs["c"], data_kwargs["deltaT"]
    r_min = I1 * c * deltaT
    r_max = I2 * c * deltaT
    result_3d, pred_histogram = CUDA_RENDERER.render_transient(
        gaussian_model=model, camera_pos=current_camera_grid_positions, theta_range=(theta_min, theta_max),
        phi_range=(phi_min, phi_max), r_range=(r_min, r_max), num_theta=args.num_sampling_points,
        num_phi=args.num_sampling_points, num_r=num_r, c=c, deltaT=deltaT, scaling_modifier=args.scaling_modifier,
        use_occlusion=args.occlusion, rendering_type=getattr(args, "rendering_type", "netf"))
    result = result_3d.reshape(num_r, args.num_sampling_points * args.num_sampling_points)
    Y = data_kwargs["volume_position"][1]
    result = result * (Y ** 2)
    pred_histogram = pred_histogram * (Y ** 2)
    return result, pred_histogram


def compute_loss(args, model, data_kwargs, optim_kwargs, device=None):
    """nlos_helpers.py:280-346 — (loss, equal_loss) for wall point (m, n)."""
    m, N, n = optim_kwargs["m"], optim_kwargs["N"], optim_kwargs["n"]
    cam = data_kwargs["camera_grid_positions"][:, m * N + n]
    with torch.no_grad():
        input_points, I1, I2, num_r, dth, dph, *_ = spherical_sample_histogram(args, data_kwargs, cam)
    result, pred = gaussian_transient_rendering(args, model, data_kwargs, input_points, cam, I1, I2, num_r, dth, dph)
    with torch.no_grad():
        target = data_kwargs["nlos_data"][I1:(I1 + num_r), m, n] * args.gt_times
    loss = optim_kwargs["criterion"](pred, target)
    equal_loss = loss / torch.mean(target ** 2)
    if getattr(args, "save_loss_mat", False):
        import scipy.io
        scipy.io.savemat("./loss_compare.mat", {"nlos": target.cpu().numpy(), "pred": pred.detach().cpu().numpy()})
    return loss, equal_loss
