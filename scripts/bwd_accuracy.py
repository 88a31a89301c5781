"""Gradient accuracy of the culled no-occlusion backward against the float64 oracle on long rays
(T bins, 5.7 sigma, cuda preset): max |err| / max |ref| per parameter.  Compare library builds with
NLOSGR_LIB (e.g. the nested-running-sum moments against the direct ones).
    python scripts/bwd_accuracy.py [T] [scale_shift]"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat
from nlosgr.geometry import build_geometry, relay_wall_grid, volume_box_point
from nlosgr.render import RenderConfig, render
from oracle import torch_ref as R
T = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
shift = float(sys.argv[2]) if len(sys.argv) > 2 else 1.2
dev = torch.device('cuda:0')
ng, ns, deg, preset, cutoff = 48, 6, 3, 'cuda', 5.7
c, deltaT = 1.0, 1.28 / T
start, end = T // 8, T // 8 + T
model = GaussianParams.synthetic(ng, deg, preset=preset, device=dev, seed=3)
with torch.no_grad():
    model._scaling.add_(shift)
walls = relay_wall_grid(2, 3, device=dev)
box = volume_box_point((0.0, 0.5, 0.0), 0.5, dev)
geo = build_geometry(walls, box, ns, start, end, c, deltaT, 0.5, preset, 'noocl')
cfg = RenderConfig(preset=preset, mode='noocl', sh_degree=deg, cutoff=cutoff, c_deltaT=c * deltaT)
hist, _ = render(model._mu, model._scaling, model._rotation, model._opacity, features_flat(model), geo, cfg)
gout = torch.randn(hist.shape, generator=torch.Generator().manual_seed(5))
(hist * gout.to(dev)).sum().backward()
d64 = lambda t: t.detach().cpu().double()
P = R.Params(d64(model._mu), d64(model._scaling), d64(model._rotation), d64(model._opacity),
             d64(model._features_dc), d64(model._features_rest), deg)
ref = R.render_volume(P, d64(walls), d64(box), 0.5, ns, start, end, c, deltaT, preset=preset, mode='noocl', mc=cutoff)
(ref * gout.double()).sum().backward()
out = {"lib": os.environ.get("NLOSGR_LIB", "default"), "T": T,
       "hist": float((hist.cpu().double() - ref.detach()).abs().max() / ref.detach().abs().max())}
for n, leaf, rleaf in zip(["mu", "scaling", "rotation", "opacity", "dc", "rest"], model.parameters(), P.leaves()):
    out[n] = float((d64(leaf.grad) - rleaf.grad).abs().max() / rleaf.grad.abs().max())
print(json.dumps(out))
