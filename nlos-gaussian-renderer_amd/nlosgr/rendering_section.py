"""Drop-in for the reference's gaussian_model/rendering_section.py on HIP.

    GaussianSectionRenderer(sigma_threshold)        (rendering_section.py:18-159)
    create_section_renderer(sigma_threshold=3.0)    (:162-176)
"""
from typing import Optional, Tuple

import torch

from .section_renderer import CUDA_AVAILABLE, SectionGaussianRendererCUDA


class GaussianSectionRenderer:
    """Thin wrapper with GaussianRendererCUDA's interface over SectionGaussianRendererCUDA."""

    def __init__(self, sigma_threshold=3.0):
        self.use_cuda = CUDA_AVAILABLE
        self.renderer = SectionGaussianRendererCUDA(sigma_threshold=sigma_threshold) if self.use_cuda else None

    def render_transient(self, gaussian_model, camera_pos: torch.Tensor, theta_range: Tuple[float, float],
                         phi_range: Tuple[float, float], r_range: Tuple[float, float], num_theta: int,
                         num_phi: int, num_r: int, c: float, deltaT: float, scaling_modifier: float = 1.0,
                         use_occlusion: bool = True, rendering_type: str = "netf"
                         ) -> Tuple[torch.Tensor, torch.Tensor]:
        if not self.use_cuda or self.renderer is None:
            raise RuntimeError("Section renderer is not available")
        return self.renderer.render_transient(gaussian_model, camera_pos, theta_range, phi_range, r_range, num_theta,
                                              num_phi, num_r, c, deltaT, scaling_modifier, use_occlusion,
                                              rendering_type)

    def render_from_spherical_samples(self, gaussian_model, input_points: torch.Tensor, camera_pos: torch.Tensor,
                                      I1: int, I2: int, num_r: int, num_angular: int, dtheta: float, dphi: float,
                                      c: float, deltaT: float, scaling_modifier: float = 1.0,
                                      use_occlusion: bool = True, rendering_type: str = "netf"
                                      ) -> Tuple[torch.Tensor, torch.Tensor]:
        if not self.use_cuda or self.renderer is None:
            raise RuntimeError("Section renderer is not available")
        return self.renderer.render_from_spherical_samples(gaussian_model, input_points, camera_pos, I1, I2, num_r,
                                                           num_angular, dtheta, dphi, c, deltaT, scaling_modifier,
                                                           use_occlusion, rendering_type)


def create_section_renderer(sigma_threshold=3.0) -> Optional[GaussianSectionRenderer]:
    """GaussianSectionRenderer when the HIP library and a GPU are available, else None."""
    if not CUDA_AVAILABLE:
        return None
    return GaussianSectionRenderer(sigma_threshold=sigma_threshold)
