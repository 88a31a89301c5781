"""Golden vectors for the space-carving initialisation, produced by running the
REFERENCE's own functions in the build container (/root/reference, read-only; the GPU box never
sees it):  gaussian_model/gaussian_utils.py  detect_first_bounces :38-49, space_carving :52-122.

Input: a synthetic confocal capture — a sphere-shaped hidden surface inside the volume, each wall
pixel's histogram a step at its round-trip bin plus a small ramp — so first bounces and carving
are non-trivial.  Output tests/golden/carving.npz: the inputs, the reference's first-bounce map and
the carved voxel coordinates.  Imports go through make_golden.import_reference.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_carving_golden.py
"""
import os
import sys
from types import SimpleNamespace

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import import_reference  # noqa: E402


def synth_capture(T=96, H=10, W=9, seed=5):
    rng = np.random.default_rng(seed)
    xs = np.linspace(-0.5, 0.5, W)
    zs = np.linspace(-0.5, 0.5, H)
    walls = np.stack([np.repeat(xs[None, :], H, 0).reshape(-1), np.zeros(H * W),
                      np.repeat(zs[:, None], W, 1).reshape(-1)]).astype(np.float32)      # [3, HW], y = 0 wall
    vol_pos = np.array([0.0, 0.5, 0.0])
    vol_size = 0.5
    deltaT, c = 1.6 / T, 1.0
    centre, radius = np.array([0.05, 0.55, -0.03]), 0.12
    data = np.zeros((T, H, W), dtype=np.float32)
    for v in range(H * W):
        y, x = divmod(v, W)
        d = np.linalg.norm(walls[:, v] - centre) - radius
        b = int(d / (c * deltaT))
        if (y + x) % 7 == 3:
            continue                                   # silent pixels (sum 0 -> no vote)
        data[b:, y, x] = 1e-3 * (1.0 + 0.1 * rng.random(T - b))
        data[:b, y, x] = 2e-6 * rng.random(b)          # sub-threshold noise before the bounce
    return data, walls, vol_pos, vol_size, deltaT, c


def main():
    gu, _shu, _GM, _H, _Config = import_reference()
    data, walls, vol_pos, vol_size, deltaT, c = synth_capture()
    fb = gu.detect_first_bounces(data[0:], threshold=1e-5)
    args = SimpleNamespace(scene="zaragoza_bunny", carving_volume_size=14, space_carving_ratio=0.6)
    data_kwargs = {
        "nlos_data": torch.from_numpy(data), "camera_grid_positions": torch.from_numpy(walls),
        "volume_position": torch.from_numpy(vol_pos).float(), "volume_size": vol_size,
        "deltaT": deltaT, "c": c,
    }
    coords2 = gu.space_carving(args, data_kwargs)
    np.savez(os.path.join(HERE, "carving.npz"), nlos_data=data, walls=walls, volume_position=vol_pos,
             volume_size=vol_size, deltaT=deltaT, c=c, carving_volume_size=args.carving_volume_size,
             space_carving_ratio=args.space_carving_ratio, first_bounces=fb, coords2=coords2.numpy())
    print("carving.npz:", fb.shape, int((fb > 0).sum()), "bounces;", coords2.shape[0], "carved voxels of",
          args.carving_volume_size ** 3)


if __name__ == "__main__":
    main()
