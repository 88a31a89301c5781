"""Backward drain / hand-off utilisation at C3 from a debug build (-DNLOSGR_BCOUNT, selected by NLOSGR_LIB):
    python scripts/bwd_counts.py [order: given|slab]"""
import ctypes, dataclasses, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat, _lib
from nlosgr.volume import Scene, make_config
from nlosgr.render import render_backward, render_forward
from nlosgr.train import slab_order
order = sys.argv[1] if len(sys.argv) > 1 else 'slab'
dev = torch.device('cuda:0')
scene = Scene(H=128, W=128, T=1024, ns=32)
m = GaussianParams.synthetic(100_000, 3, preset='cuda', device=dev, seed=0)
geo = scene.geometry(dev, 'cuda')
args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), features_flat(m).detach(), geo)
if order == 'slab':
    perm = slab_order(args[0], geo.wall, size=args[1].max(1).values)
    args = tuple(t[perm].contiguous() for t in args[:5]) + (geo,)
cfg = make_config(m, scene, 'cuda', cutoff=5.7)
hist = render_forward(*args, cfg)[0]
grad = torch.randn_like(hist) * 1e-3
lib = _lib.load()
f = lib.nlosgr_debug_bwd_counts
f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 8)()
torch.cuda.synchronize(); f(buf)
render_backward(*args, cfg, grad_hist=grad)
torch.cuda.synchronize(); f(buf)
c = list(buf)
print(json.dumps({"order": order, "iterations": c[0], "drain_rounds": c[1], "active_per_drain_round": c[2] / max(c[1], 1),
                  "handoff_rounds": c[3], "pending_per_handoff_round": c[4] / max(c[3], 1),
                  "handoffs_per_handoff_round": c[5] / max(c[3], 1), "refills": c[6], "taken_per_refill": c[7] / max(c[6], 1)}))
