import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat
from nlosgr.volume import Scene, make_config
from nlosgr.render import render_forward
dev = torch.device('cuda:0')
scene = Scene(H=8, W=8, T=256, ns=32)
m = GaussianParams.synthetic(2000, 3, preset="cuda", device=dev, seed=1)
geo = scene.geometry(dev, "cuda")
f = features_flat(m).detach()
cd, c6 = make_config(m, scene, cutoff=0.0), make_config(m, scene, cutoff=6.0)
rows = []
with torch.no_grad():
    for g in range(2000):
        sl = slice(g, g + 1)
        args = (m._mu[sl], m._scaling[sl], m._rotation[sl], m._opacity[sl], f[sl], geo)
        hd, _ = render_forward(*args, cd)
        h6, _ = render_forward(*args, c6)
        rows.append(((hd - h6).abs().sum() / hd.abs().sum().clamp_min(1e-30)).item())
rows = torch.tensor(rows)
idx = rows.argsort(descending=True)[:10]
print('per-gaussian rel L1 diff: max', rows.max().item(), 'median', rows.median().item())
for g in idx.tolist():
    print(g, rows[g].item(), 'mu', m._mu[g].tolist(), 'scal', m._scaling[g].tolist(), 'rot', m._rotation[g].tolist())
