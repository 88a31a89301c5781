"""Backward wall-split sweep at C3 (RenderConfig.nsplit; 0 = automatic): one timed ray-cache backward each."""
import dataclasses, os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat
from nlosgr.volume import Scene, make_config
from nlosgr.render import render_backward, render_forward
dev = torch.device('cuda:0')
scene = Scene(H=128, W=128, T=1024, ns=32)
m = GaussianParams.synthetic(100_000, 3, preset="cuda", device=dev, seed=0)
geo = scene.geometry(dev, "cuda")
args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), features_flat(m).detach(), geo)
base = make_config(m, scene, cutoff=3.0)
res = {}
for ns in [int(x) for x in (sys.argv[1:] or ["0", "1", "3", "4", "8", "16"])]:
    cfg = dataclasses.replace(base, nsplit=ns)
    hist, _, ws = render_forward(*args, cfg, ray_cache=True)
    grad = torch.randn_like(hist) * 1e-3
    render_backward(*args, cfg, grad_hist=grad, workspace=ws, ray_cache=True); torch.cuda.synchronize()
    t0 = time.perf_counter(); render_backward(*args, cfg, grad_hist=grad, workspace=ws, ray_cache=True); torch.cuda.synchronize()
    res[ns] = round((time.perf_counter() - t0) * 1000, 1)
    del ws
print(json.dumps({"bwd_ms_by_nsplit": res}))
