"""Backward wall-point splits (opt.nsplit, 0 = the library's ~48k-workgroup target) at C3, timed
without the ray cache: median of 3 after one warm-up per value.
    python scripts/nsplit_sweep.py [cutoff] [nsplit ...]"""
import sys, os, time, json, statistics
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch, dataclasses
from nlosgr import GaussianParams, features_flat
from nlosgr.volume import Scene, make_config
from nlosgr.render import render_backward, render_forward

cutoff = float(sys.argv[1]) if len(sys.argv) > 1 else 5.7
values = [int(v) for v in sys.argv[2:]] or [0, 8, 16, 32, 64]
dev = torch.device('cuda:0')
scene = Scene(H=128, W=128, T=1024, ns=32)
m = GaussianParams.synthetic(100_000, 3, preset='cuda', device=dev, seed=0)
geo = scene.geometry(dev, 'cuda')
f = features_flat(m).detach()
args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), f, geo)
base = make_config(m, scene, 'cuda', cutoff=cutoff)
hist = render_forward(*args, base)[0]
grad = torch.randn_like(hist) * 1e-3
out = {}
for ns in values:
    cfg = dataclasses.replace(base, nsplit=ns)
    render_backward(*args, cfg, grad_hist=grad); torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter(); render_backward(*args, cfg, grad_hist=grad); torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1000)
    out[ns] = round(statistics.median(ts), 1)
    print(ns, out[ns], flush=True)
print(json.dumps({'cutoff': cutoff, 'bwd_ms_by_nsplit': out}))
