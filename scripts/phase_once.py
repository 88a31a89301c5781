"""One C3 forward and one ray-cache backward with the given diagnostic flags (for PMC passes):
    python scripts/phase_once.py [fwd_flags] [bwd_flags] [config]"""
import dataclasses, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat
from nlosgr.volume import Scene, make_config
from nlosgr.render import render_backward, render_forward
ff = int(sys.argv[1]) if len(sys.argv) > 1 else 0
bf = int(sys.argv[2]) if len(sys.argv) > 2 else 0
cfgname = sys.argv[3] if len(sys.argv) > 3 else 'C3'
ng, H, T = {'C3': (100_000, 128, 1024), 'S1': (20_000, 32, 512)}[cfgname]
dev = torch.device('cuda:0')
scene = Scene(H=H, W=H, T=T, ns=32)
m = GaussianParams.synthetic(ng, 3, preset="cuda", device=dev, seed=0)
geo = scene.geometry(dev, "cuda")
args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), features_flat(m).detach(), geo)
base = make_config(m, scene, cutoff=float(os.environ.get("PHASE_CUTOFF", "3.0")))
ray_cache = os.environ.get("PHASE_CACHE", "1") == "1"
out = render_forward(*args, dataclasses.replace(base, flags=ff), ray_cache=ray_cache)
hist, ws = out[0], (out[2] if ray_cache else None)
grad = torch.randn_like(hist) * 1e-3
render_backward(*args, dataclasses.replace(base, flags=bf), grad_hist=grad, workspace=ws, ray_cache=ray_cache)
torch.cuda.synchronize()
print("done", ff, bf)
