"""Space-carving initialisation on CPU: the oracle restatement (oracle/carving.py) and the torch
first-bounce detector against the reference's own outputs (tests/golden/carving.npz, made by
tests/golden/make_carving_golden.py from gaussian_utils.py:38-122)."""
import os

import numpy as np
import torch

from conftest import GOLDEN


def _golden():
    return np.load(os.path.join(GOLDEN, "carving.npz"), allow_pickle=False)


def test_oracle_first_bounces_match_reference():
    from oracle.carving import first_bounces
    z = _golden()
    np.testing.assert_array_equal(first_bounces(z["nlos_data"]), z["first_bounces"])


def test_torch_first_bounces_match_reference():
    from nlosgr.init import detect_first_bounces
    z = _golden()
    np.testing.assert_array_equal(detect_first_bounces(z["nlos_data"]), z["first_bounces"])
    t = detect_first_bounces(torch.from_numpy(z["nlos_data"]))
    np.testing.assert_array_equal(t.numpy(), z["first_bounces"].astype(np.float32))


def test_oracle_space_carving_matches_reference():
    from oracle.carving import space_carving
    z = _golden()
    got = space_carving(z["nlos_data"], z["walls"], z["volume_position"], float(z["volume_size"]), float(z["c"]),
                        float(z["deltaT"]), int(z["carving_volume_size"]), float(z["space_carving_ratio"]))[0]
    np.testing.assert_allclose(got, z["coords2"], rtol=0, atol=1e-6)
