"""Gaussian parameter container with the reference GaussianModel's attribute names.

The renderer reads only these attributes (gaussian_model/gaussian_model.py:38-49, :107-135),
so the reference's own GaussianModel works as-is; GaussianParams is the minimal stand-in used
by the benchmark, the tests and the multi-GPU driver.  Optimisation state, densification and
initialisation heuristics of the reference are out of scope.
"""
import math

import torch
import torch.nn as nn

SH_C0 = 0.28209479177387814


def features_flat(model):
    """[Ng, K] = cat(_features_dc, _features_rest) flattened (gaussian_model.py:120-123)."""
    dc = model._features_dc
    rest = model._features_rest
    ng = dc.shape[0]
    return torch.cat((dc.reshape(ng, -1), rest.reshape(ng, -1)), dim=1)


class GaussianParams:
    def __init__(self, mu, scaling, rotation, opacity, features_dc, features_rest, active_sh_degree=0,
                 max_sh_degree=None):
        self._mu = nn.Parameter(mu)
        self._scaling = nn.Parameter(scaling)
        self._rotation = nn.Parameter(rotation)
        self._opacity = nn.Parameter(opacity)
        self._features_dc = nn.Parameter(features_dc)
        self._features_rest = nn.Parameter(features_rest)
        K = features_dc.shape[1] * features_dc.shape[2] + features_rest.shape[1] * features_rest.shape[2]
        self.max_sh_degree = int(round(math.sqrt(K))) - 1 if max_sh_degree is None else max_sh_degree
        self.active_sh_degree = int(active_sh_degree)

    # --- reference property surface (gaussian_model.py:107-135) ---
    @property
    def get_mu(self):
        return self._mu

    @property
    def get_scaling(self):
        return torch.exp(self._scaling)

    @property
    def get_rotation(self):
        return torch.nn.functional.normalize(self._rotation)

    @property
    def get_opacity(self):
        return torch.sigmoid(self._opacity)

    @property
    def get_features(self):
        return torch.cat((self._features_dc, self._features_rest), dim=1)

    @property
    def get_features_dc(self):
        return self._features_dc

    @property
    def get_features_rest(self):
        return self._features_rest

    def parameters(self):
        return [self._mu, self._scaling, self._rotation, self._opacity, self._features_dc, self._features_rest]

    def oneupSHdegree(self):
        if self.active_sh_degree < self.max_sh_degree:
            self.active_sh_degree += 1

    def state_dict(self):
        """Checkpoint dict with the reference's keys (gaussian_model.py:63-74) minus the pickled
        optimizer object (safe to load with torch.load(weights_only=True))."""
        return {"mu": self._mu.detach(), "features_dc": self._features_dc.detach(),
                "features_rest": self._features_rest.detach(), "opacity": self._opacity.detach(),
                "scaling": self._scaling.detach(), "rotation": self._rotation.detach(),
                "max_sh_degree": self.max_sh_degree, "active_sh_degree": self.active_sh_degree}

    @classmethod
    def from_state_dict(cls, d, device=None):
        t = lambda k: d[k].detach().float().to(device).clone()
        return cls(t("mu"), t("scaling"), t("rotation"), t("opacity"), t("features_dc"), t("features_rest"),
                   d.get("active_sh_degree", 0), d.get("max_sh_degree"))

    @classmethod
    def synthetic(cls, ng, sh_degree=3, preset="cuda", device=None, seed=0, volume_position=(0.0, 0.5, 0.0),
                  volume_size=0.5, margin=0.1):
        """SURVEY §8d synthetic Gaussians: mu ~ U(box shrunk by margin, gaussian_utils.py:28-30),
        rotation ~ N(0,1)^4, opacity ~ N(0,1), dc = RHO2SH(U(0,0.2)) (main.py:77, sh_utils.py:114),
        rest ~ 0.05 N(0,1); log-scale log(0.5/Ng^(1/3)) + 0.2 N(0,1) under the cuda preset (the torch
        preset's double exp makes every std >= 1, so its scales are drawn as N(-1, 0.7))."""
        g = torch.Generator().manual_seed(seed)
        c = torch.tensor(volume_position, dtype=torch.float32)
        pmin, pmax = c - volume_size / 2, c + volume_size / 2
        lo = pmin + (pmin * margin).abs()
        hi = pmax - (pmax * margin).abs()
        mu = torch.rand(ng, 3, generator=g) * (hi - lo) + lo
        K = (sh_degree + 1) ** 2
        if preset == "cuda":
            scaling = math.log(0.5 / ng ** (1.0 / 3.0)) + 0.2 * torch.randn(ng, 3, generator=g)
        else:
            scaling = torch.randn(ng, 3, generator=g) * 0.7 - 1.0
        rotation = torch.randn(ng, 4, generator=g)
        opacity = torch.randn(ng, 1, generator=g)
        rho = torch.rand(ng, 1, generator=g) * 0.2
        fdc = ((rho - 0.5) / SH_C0).reshape(ng, 1, 1)
        frest = 0.05 * torch.randn(ng, K - 1, 1, generator=g)
        dev = lambda t: t.float().to(device).contiguous()
        return cls(dev(mu), dev(scaling), dev(rotation), dev(opacity), dev(fdc), dev(frest), sh_degree, sh_degree)
