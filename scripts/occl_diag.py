"""Per-phase cycles of the ray-tile engine (diagnostic build ab/diag.so, NLOSGR_TILES_DIAG=1) for one
wall-point batch of C3 with path C occlusion / AABB selection: forward (rows cached) and backward.
    python scripts/occl_diag.py [mode] [selection] [nobin]   (nobin: in-kernel cull, FLAG_TILE_NOBIN)"""
import os, sys, dataclasses
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat
from nlosgr.volume import Scene, make_config
from nlosgr.render import render_backward, render_forward
mode = sys.argv[1] if len(sys.argv) > 1 else 'occl'
sel = sys.argv[2] if len(sys.argv) > 2 else 'aabb'
dev = torch.device('cuda:0')
scene = Scene(H=128, W=128, T=1024, ns=32)
m = GaussianParams.synthetic(100_000, 3, preset='cuda', device=dev, seed=0)
geo = scene.geometry(dev, 'cuda', mode).slice(4096, 5120)
cfg = make_config(m, scene, 'cuda', mode, cutoff=5.7, selection=sel)
if 'nobin' in sys.argv[3:]:
    from nlosgr import _lib
    cfg = dataclasses.replace(cfg, flags=_lib.FLAG_TILE_NOBIN)
args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), features_flat(m).detach())
os.environ['NLOSGR_TILES_DIAG'] = '1'
h, _, ws = render_forward(*args, geo, cfg, ray_cache=True)
render_backward(*args, geo, cfg, grad_hist=torch.ones_like(h) * 1e-3, workspace=ws, ray_cache=True)
torch.cuda.synchronize()
