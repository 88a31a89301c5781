"""Space-carving vote throughput: nlosgr_carve_votes on the GPU at the reference's
realistic size (256x256 wall points, carving grid N^3) vs the oracle's per-wall-point loop (the
reference's structure, gaussian_utils.py:88-99) timed on a bounded sample of wall points on the host
and extrapolated.  Prints one JSON line.   python scripts/bench_carving.py [N=128] [H=256]"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlos-gaussian-renderer_amd")); sys.path.insert(0, ROOT)
import numpy as np
import torch
from nlosgr.init import carve_votes
from oracle.carving import carve_votes as carve_ref

N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
H = int(sys.argv[2]) if len(sys.argv) > 2 else 256
dev = torch.device("cuda:0")
axis = np.linspace(-0.25, 0.25, N)
coords = np.stack(np.meshgrid(axis, axis, axis, indexing="ij"), -1).reshape(-1, 3).astype(np.float32)
xs = np.linspace(-0.5, 0.5, H)
walls = np.stack([np.repeat(xs[None], H, 0).reshape(-1), np.full(H * H, -0.5), np.repeat(xs[:, None], H, 1).reshape(-1)],
                 -1).astype(np.float32)
radii = (0.3 + 0.1 * np.random.default_rng(0).random(H * H)).astype(np.float32)
c, w, r = (torch.from_numpy(a).to(dev) for a in (coords, walls, radii))
carve_votes(c, w, r)
torch.cuda.synchronize()
t0 = time.perf_counter()
reps = 3
for _ in range(reps):
    votes = carve_votes(c, w, r)
torch.cuda.synchronize()
gpu_s = (time.perf_counter() - t0) / reps
tests = coords.shape[0] * walls.shape[0]
ms = 16
t0 = time.perf_counter()
ref = carve_ref(coords, walls[:ms], radii[:ms])
cpu_s = (time.perf_counter() - t0) * walls.shape[0] / ms
assert (carve_votes(c, w[:ms], r[:ms]).cpu().numpy() == ref).all()
flop = 9 * tests   # 3 sub, 3 mul, 2 add, 1 sqrt per voxel x wall-point test
print(json.dumps({"workload": f"{N}^3 voxels x {H}x{H} wall points", "tests": tests, "gpu_ms": gpu_s * 1e3,
                  "tests_per_s": tests / gpu_s, "valu_tflops": flop / gpu_s / 1e12, "valu_frac": flop / gpu_s / 157.3e12,
                  "cpu_ref_loop_s_extrapolated": cpu_s, "cpu_sample": f"{ms} wall points, numpy, 1 process",
                  "speedup": cpu_s / gpu_s}))
