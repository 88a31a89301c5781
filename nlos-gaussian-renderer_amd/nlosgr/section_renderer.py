"""Drop-in for the reference's submodules/cuda_renderer/section_renderer.py (path A, the
"analytic" section renderer) on HIP.

    CUDA_AVAILABLE                                          (section_renderer.py:13-18)
    SectionGaussianRendererCUDA(sigma_threshold)            (:21-288)
        .render_transient(...)                              (:55-186)
        .render_from_spherical_samples(...)                 (:188-260)
        .filter_gaussians(...)                              (:262-288)
    create_section_renderer(sigma_threshold=3.0)            (:291-305)

Behaviour is the reference's, including what it does with the result: one value per ray
(nlosgr_rays_analytic), placed in the middle radial bin of `result`, and a histogram that is the
angular sum broadcast to every bin (:171-184).  Boxes are the GaussianModel.get_bboxes boxes
(gaussian_model.py:140-178), computed by nlosgr_bboxes (preset "torch": single exp, doubly
normalised quaternion, 1e-8 clamp) so any model exposing the raw tensors works.  Only the dc
features are passed, as in the reference (:121,139); SH is evaluated up to the degree the feature
row supports (the reference reads past the row when active_sh_degree > 0 — not reproduced).
"""
from typing import Optional, Tuple

import torch

from . import _lib
from .rays import filter_gaussians_per_ray, render_rays_analytic
from .render import bboxes

CUDA_AVAILABLE = _lib.available()


class SectionGaussianRendererCUDA:
    """Section-based renderer with the reference's API (see module docstring)."""

    def __init__(self, sigma_threshold=3.0):
        if not CUDA_AVAILABLE:
            raise RuntimeError("HIP renderer is not available (libnlosgr.so / GPU missing). "
                               "Cannot use SectionGaussianRendererCUDA.")
        self.sigma_threshold = sigma_threshold

    def render_transient(self, gaussian_model, camera_pos: torch.Tensor, theta_range: Tuple[float, float],
                         phi_range: Tuple[float, float], r_range: Tuple[float, float], num_theta: int,
                         num_phi: int, num_r: int, c: float, deltaT: float, scaling_modifier: float = 1.0,
                         use_occlusion: bool = True, rendering_type: str = "netf"
                         ) -> Tuple[torch.Tensor, torch.Tensor]:
        """result [num_r, num_theta, num_phi] (middle bin only), pred_histogram [num_r]."""
        device = camera_pos.device
        theta = torch.linspace(theta_range[0], theta_range[1], num_theta, device=device)
        phi = torch.linspace(phi_range[0], phi_range[1], num_phi, device=device)
        theta_grid, phi_grid = torch.meshgrid(theta, phi, indexing="ij")
        tf, pf = theta_grid.reshape(-1), phi_grid.reshape(-1)
        ray_dirs = torch.stack([torch.sin(tf) * torch.cos(pf), torch.sin(tf) * torch.sin(pf), torch.cos(tf)], dim=1)
        ray_origins = camera_pos.unsqueeze(0).expand(tf.shape[0], 3).contiguous()
        means = gaussian_model.get_mu
        bb = bboxes(means, gaussian_model._scaling, gaussian_model._rotation, scaling_modifier,
                    self.sigma_threshold, preset="torch")
        filt = filter_gaussians_per_ray(ray_origins, ray_dirs.contiguous(), means, bb.view(-1, 6),
                                        self.sigma_threshold)
        sh_features = gaussian_model.get_features_dc.reshape(means.shape[0], -1)
        histogram = render_rays_analytic(ray_origins, ray_dirs.contiguous(), r_range[0], r_range[1], filt, means,
                                         gaussian_model._scaling, gaussian_model._rotation,
                                         gaussian_model._opacity, sh_features, camera_pos,
                                         gaussian_model.active_sh_degree, c, deltaT, scaling_modifier,
                                         self.sigma_threshold, rendering_type)
        histogram_2d = histogram.reshape(num_theta, num_phi)
        result = torch.zeros(num_r, num_theta, num_phi, device=device)
        result[num_r // 2] = histogram_2d
        dtheta = (theta_range[1] - theta_range[0]) / num_theta
        dphi = (phi_range[1] - phi_range[0]) / num_phi
        pred_histogram = (torch.sum(histogram_2d) * dtheta * dphi).expand(num_r)
        return result, pred_histogram

    def render_from_spherical_samples(self, gaussian_model, input_points: torch.Tensor, camera_pos: torch.Tensor,
                                      I1: int, I2: int, num_r: int, num_angular: int, dtheta: float, dphi: float,
                                      c: float, deltaT: float, scaling_modifier: float = 1.0,
                                      use_occlusion: bool = True, rendering_type: str = "netf"
                                      ) -> Tuple[torch.Tensor, torch.Tensor]:
        """Angular ranges recovered from spherical_sample_histogram's input_points (:228-238);
        result [num_r, num_angular^2], pred_histogram [num_r]."""
        theta_vals, phi_vals = input_points[:, 3], input_points[:, 4]
        theta_range = (theta_vals.min().item(), theta_vals.max().item())
        phi_range = (phi_vals.min().item(), phi_vals.max().item())
        r_range = (I1 * c * deltaT, I2 * c * deltaT)
        result_3d, pred_histogram = self.render_transient(gaussian_model, camera_pos, theta_range, phi_range,
                                                          r_range, num_angular, num_angular, num_r, c, deltaT,
                                                          scaling_modifier, use_occlusion, rendering_type)
        return result_3d.reshape(num_r, num_angular * num_angular), pred_histogram

    def filter_gaussians(self, ray_origins, ray_directions, gaussian_means, gaussian_bboxes):
        """[N_rays, 257] int32: count, first 256 hits by index, -1 padding (:262-288)."""
        return filter_gaussians_per_ray(ray_origins, ray_directions, gaussian_means,
                                        gaussian_bboxes.reshape(-1, 6), self.sigma_threshold)


def create_section_renderer(sigma_threshold=3.0) -> Optional[SectionGaussianRendererCUDA]:
    """SectionGaussianRendererCUDA when the HIP library and a GPU are available, else None."""
    if not CUDA_AVAILABLE:
        return None
    return SectionGaussianRendererCUDA(sigma_threshold=sigma_threshold)
