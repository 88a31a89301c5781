"""Drop-in for the reference's gaussian_model/rendering_cuda.py on HIP.

    CUDA_AVAILABLE                                  (rendering_cuda.py:10-15)
    GaussianRendererCUDA(sigma_threshold)           (:188-336)
        .render_transient(...)                      (:208-263)
        .render_from_spherical_samples(...)         (:265-336)
    create_cuda_renderer(sigma_threshold=3.0)       (:339-353)
"""
from typing import Optional, Tuple

import torch

from .cuda_autograd import CUDA_AVAILABLE, CUDARenderModule, create_cuda_render_module  # noqa: F401


class GaussianRendererCUDA:
    """Ray-based renderer with the reference's render API (path C conventions, real gradients)."""

    def __init__(self, sigma_threshold=3.0):
        self.use_cuda = CUDA_AVAILABLE
        self.renderer = CUDARenderModule(sigma_threshold=sigma_threshold) if self.use_cuda else None

    def render_transient(self, gaussian_model, camera_pos: torch.Tensor, theta_range: Tuple[float, float],
                         phi_range: Tuple[float, float], r_range: Tuple[float, float], num_theta: int,
                         num_phi: int, num_r: int, c: float, deltaT: float, scaling_modifier: float = 1.0,
                         use_occlusion: bool = True, rendering_type: str = "netf"
                         ) -> Tuple[torch.Tensor, torch.Tensor]:
        """result [num_r, num_theta, num_phi], pred_histogram [num_r]."""
        if not self.use_cuda or self.renderer is None:
            raise RuntimeError("CUDA renderer is not available")
        return self.renderer(gaussian_model=gaussian_model, camera_pos=camera_pos, theta_range=theta_range,
                             phi_range=phi_range, r_range=r_range, num_theta=num_theta, num_phi=num_phi,
                             num_r=num_r, c=c, deltaT=deltaT, scaling_modifier=scaling_modifier,
                             use_occlusion=use_occlusion, rendering_type=rendering_type)

    def render_from_spherical_samples(self, gaussian_model, input_points: torch.Tensor, camera_pos: torch.Tensor,
                                      I1: int, I2: int, num_r: int, num_angular: int, dtheta: float, dphi: float,
                                      c: float, deltaT: float, scaling_modifier: float = 1.0,
                                      use_occlusion: bool = True, rendering_type: str = "netf"
                                      ) -> Tuple[torch.Tensor, torch.Tensor]:
        """Angular ranges recovered from spherical_sample_histogram's input_points; result
        [num_r, num_angular^2], pred_histogram [num_r]."""
        theta_vals, phi_vals = input_points[:, 3], input_points[:, 4]
        theta_range = (theta_vals.min().item(), theta_vals.max().item())
        phi_range = (phi_vals.min().item(), phi_vals.max().item())
        r_range = (I1 * c * deltaT, I2 * c * deltaT)
        result_3d, pred_histogram = self.render_transient(gaussian_model, camera_pos, theta_range, phi_range, r_range,
                                                          num_angular, num_angular, num_r, c, deltaT,
                                                          scaling_modifier, use_occlusion, rendering_type)
        return result_3d.reshape(num_r, num_angular * num_angular), pred_histogram


def create_cuda_renderer(sigma_threshold=3.0) -> Optional[GaussianRendererCUDA]:
    """GaussianRendererCUDA when the HIP library and a GPU are available, else None."""
    if not CUDA_AVAILABLE:
        return None
    return GaussianRendererCUDA(sigma_threshold=sigma_threshold)
