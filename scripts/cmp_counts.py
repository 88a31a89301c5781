"""Support counts and culled-vs-dense errors of the loaded library (NLOSGR_LIB selects an A/B build):
the cutoff-convergence scene of tests/test_gpu_parity.py plus C3-sized counts."""
import sys, os, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat
from nlosgr.volume import Scene, make_config, render_volume
from nlosgr.render import count_support
dev = torch.device('cuda:0')
out = {}
scene = Scene(H=8, W=8, T=256, ns=32)
model = GaussianParams.synthetic(2000, 3, preset="cuda", device=dev, seed=1)
geo = scene.geometry(dev, "cuda")
params = [model._mu.detach(), model._scaling.detach(), model._rotation.detach(), model._opacity.detach(),
          features_flat(model).detach().contiguous()]
with torch.no_grad():
    dense = render_volume(model, geo, make_config(model, scene, cutoff=0.0))
    for mc in (3.0, 4.0, 5.0, 6.0):
        cfg = make_config(model, scene, cutoff=mc)
        h = render_volume(model, geo, cfg)
        out[f"small_mc{mc}"] = {"err": ((h - dense).norm() / dense.norm()).item(),
                                "counts": list(count_support(*params, geo, cfg))}
scene = Scene(H=128, W=128, T=1024, ns=32)
model = GaussianParams.synthetic(100_000, 3, preset="cuda", device=dev, seed=0)
geo = scene.geometry(dev, "cuda")
params = [model._mu.detach(), model._scaling.detach(), model._rotation.detach(), model._opacity.detach(),
          features_flat(model).detach().contiguous()]
out["C3"] = list(count_support(*params, geo, make_config(model, scene, cutoff=3.0)))
print(json.dumps(out))
