"""Diagnostic (GPU): per-Gaussian check of the sweep forward against the lane-serial drain: renders
single Gaussians (one at a time) at 3x3 wall points and prints the sum ratio per Gaussian."""
import os, sys
from dataclasses import replace
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlos-gaussian-renderer_amd")); sys.path.insert(0, ROOT)
from nlosgr import GaussianParams, features_flat
from nlosgr.render import render_forward
from nlosgr.volume import Scene, make_config
dev = torch.device("cuda:0")
scene = Scene(H=3, W=3, T=1024, ns=32)
m = GaussianParams.synthetic(6000, 3, preset="cuda", device=dev, seed=21)
geo = scene.geometry(dev, "cuda")
full = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), features_flat(m).detach().contiguous())
cfg = make_config(m, scene, "cuda", cutoff=5.7)
for ng in (1, 64, 1000):
    rs = []
    for g0 in range(0, min(6000, 6 * ng), ng):
        args = tuple(t[g0:g0 + ng].contiguous() for t in full) + (geo,)
        os.environ["NLOSGR_FSWEEP"] = "1"
        sw, _ = render_forward(*args, cfg)
        os.environ["NLOSGR_FSWEEP"] = "0"
        ls, _ = render_forward(*args, cfg)
        os.environ.pop("NLOSGR_FSWEEP", None)
        if ls.sum() > 0:
            rs.append((sw.sum() / ls.sum() - 1).item())
    print(f"ng {ng}: sum ratio - 1 per chunk: {', '.join(f'{r:.2e}' for r in rs)}", flush=True)
# accumulation check: the lane-serial histogram of all 6000 Gaussians vs the float64 sum of its
# histograms over 24 chunks of 250 (each chunk's running fp32 totals are 24x smaller)
args = full + (geo,)
os.environ["NLOSGR_FSWEEP"] = "1"
sw, _ = render_forward(*args, cfg)
os.environ["NLOSGR_FSWEEP"] = "0"
ls, _ = render_forward(*args, cfg)
parts = torch.zeros_like(ls, dtype=torch.float64)
sparts = torch.zeros_like(ls, dtype=torch.float64)
for g0 in range(0, 6000, 250):
    a = tuple(t[g0:g0 + 250].contiguous() for t in full) + (geo,)
    os.environ["NLOSGR_FSWEEP"] = "0"
    parts += render_forward(*a, cfg)[0].double()
    os.environ["NLOSGR_FSWEEP"] = "1"
    sparts += render_forward(*a, cfg)[0].double()
os.environ.pop("NLOSGR_FSWEEP", None)
rel = lambda x, y: ((x.double() - y).norm() / y.norm()).item()
print(f"vs float64 sum of 24 lane-serial parts: lane-serial {rel(ls, parts):.2e} sweep {rel(sw, parts):.2e}; "
      f"sweep parts vs ls parts {rel(sparts, parts):.2e}", flush=True)
