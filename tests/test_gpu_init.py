"""GPU space-carving initialisation (nlosgr_carve_votes through the C ABI) against the oracle and
the reference's own carved voxels (tests/golden/carving.npz): integer votes bit-exact, carved set
identical; sampling helpers keep the reference's bounds."""
import os
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _golden():
    return np.load(os.path.join(GOLDEN, "carving.npz"), allow_pickle=False)


def _data_kwargs(z, dev):
    vp = torch.from_numpy(z["volume_position"]).float().to(dev)
    vs = float(z["volume_size"])
    pmin = torch.cat([vp - vs / 2, torch.tensor([0.0, -np.pi], device=dev)])
    pmax = torch.cat([vp + vs / 2, torch.tensor([np.pi, 0.0], device=dev)])
    return {"nlos_data": torch.from_numpy(z["nlos_data"]).to(dev),
            "camera_grid_positions": torch.from_numpy(z["walls"]).to(dev), "volume_position": vp,
            "volume_size": vs, "deltaT": float(z["deltaT"]), "c": float(z["c"]), "pmin": pmin, "pmax": pmax}


def test_carve_votes_match_oracle():
    from nlosgr.init import carve_votes
    from oracle.carving import space_carving as ref
    z = _golden()
    _, votes, coords, walls, radii = ref(z["nlos_data"], z["walls"], z["volume_position"], float(z["volume_size"]),
                                        float(z["c"]), float(z["deltaT"]), int(z["carving_volume_size"]),
                                        float(z["space_carving_ratio"]))
    dev = torch.device("cuda:0")
    got = carve_votes(torch.from_numpy(coords).to(dev), torch.from_numpy(walls).to(dev),
                      torch.from_numpy(radii.astype(np.float32)).to(dev))
    np.testing.assert_array_equal(got.cpu().numpy(), votes)


def test_space_carving_matches_reference():
    from nlosgr.init import space_carving
    z = _golden()
    dev = torch.device("cuda:0")
    args = SimpleNamespace(carving_volume_size=int(z["carving_volume_size"]),
                           space_carving_ratio=float(z["space_carving_ratio"]))
    got = space_carving(args, _data_kwargs(z, dev)).cpu().numpy()
    np.testing.assert_allclose(got, z["coords2"], rtol=0, atol=1e-6)


def test_sampling_helpers_bounds():
    from nlosgr.init import init_rand_points, sample_from_feasible_space_jittering
    z = _golden()
    dev = torch.device("cuda:0")
    dk = _data_kwargs(z, dev)
    n = int(z["carving_volume_size"])
    args = SimpleNamespace(init_gaussian_num=500, carving_volume_size=n, space_carving_ratio=float(z["space_carving_ratio"]))
    np.random.seed(0)
    torch.manual_seed(0)
    pts, rho = sample_from_feasible_space_jittering(args, dk, rho_scale=0.2)
    assert pts.shape == (500, 3) and rho.shape == (500, 1) and (0 <= rho).all() and (rho <= 0.2).all()
    carved = torch.from_numpy(z["coords2"]).to(dev)
    half = float(z["volume_size"]) / (n - 1) / 2
    dist = (pts[:, None, :] - carved[None]).abs().amax(-1).amin(1)     # Chebyshev distance to a carved voxel
    assert (dist <= half + 1e-5).all()
    samples, rho2 = init_rand_points(args, dk, margin=0.1, rho_scale=0.2)
    lo = dk["pmin"][:3].cpu().numpy()
    hi = dk["pmax"][:3].cpu().numpy()
    assert samples.shape == (500, 3) and (samples >= lo + np.abs(lo * 0.1) - 1e-6).all()
    assert (samples <= hi - np.abs(hi * 0.1) + 1e-6).all()


def test_carve_votes_rejects_cpu_tensors():
    from nlosgr.init import carve_votes
    with pytest.raises(RuntimeError):
        carve_votes(torch.zeros(4, 3), torch.zeros(2, 3), torch.ones(2))
