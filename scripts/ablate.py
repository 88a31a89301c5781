"""Ablation timing of the forward / backward kernel phases (diagnostic opt.flags bits:
2 = pair setup only, 1 = + candidate enumeration, 4 = + segment records, 0 = everything)."""
import sys, os, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch, dataclasses
from nlosgr import GaussianParams, features_flat
from nlosgr.volume import Scene, make_config
from nlosgr.render import render_backward, render_forward
cfgname = sys.argv[1] if len(sys.argv) > 1 else 'C3'
sizes = {'C3': (100_000, 128, 1024), 'S1': (20_000, 32, 512), 'C5B': (500_000, 256, 2048), 'C1': (1_000, 32, 128)}
preset = os.environ.get('NLOSGR_ABLATE_PRESET', 'cuda')
cutoff = float(os.environ.get('NLOSGR_ABLATE_CUTOFF', '3.0'))
mode = os.environ.get('NLOSGR_ABLATE_MODE', 'noocl')
ng, H, T = sizes[cfgname]
dev = torch.device('cuda:0')
scene = Scene(H=H, W=H, T=T, ns=32)
m = GaussianParams.synthetic(ng, 3, preset=preset, device=dev, seed=0)
if cfgname == 'C5B':   # one rank's band of the 8-way C5 wall shard
    from nlosgr.distributed import wall_band
    b0, b1 = wall_band(H * H, 0, 8)
    geo = scene.geometry(dev, preset, walls=scene.walls(dev)[b0:b1].contiguous())
else:
    geo = scene.geometry(dev, preset, mode)
f = features_flat(m).detach()
args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), f, geo)
if os.environ.get('NLOSGR_ABLATE_ORDER') == 'slab':   # the Gaussian order TrainStep hands the backward
    from nlosgr.train import slab_order, wall_centroid
    perm = slab_order(args[0], None, 8, 4, size=args[1].max(1).values, centroid=wall_centroid(geo.wall))
    args = tuple(t[perm].contiguous() for t in args[:5]) + (geo,)
base = make_config(m, scene, preset, mode, cutoff=cutoff)
res = {}
for flags in (0, 4, 1, 2):
    cfg = dataclasses.replace(base, flags=flags)
    render_forward(*args, cfg); torch.cuda.synchronize()
    t0 = time.perf_counter(); render_forward(*args, cfg); torch.cuda.synchronize()
    res[flags] = (time.perf_counter() - t0) * 1000
if os.environ.get("NLOSGR_ABLATE_FWD_ONLY") == "1":
    print(json.dumps({'config': cfgname, 'mode': mode, 'cutoff': cutoff, 'fwd_ms_by_flags': res}))
    sys.exit(0)
cache = os.environ.get("NLOSGR_ABLATE_CACHE", "1") == "1"
if cache:
    hist, _, ws = render_forward(*args, base, ray_cache=True)
else:
    hist, _ = render_forward(*args, base)
grad = torch.randn_like(hist) * 1e-3
bres = {}
for flags in (0, 64, 32, 4, 1, 2):
    cfg = dataclasses.replace(base, flags=flags)
    kw = dict(workspace=ws, ray_cache=True) if cache else {}
    render_backward(*args, cfg, grad_hist=grad, **kw); torch.cuda.synchronize()
    t0 = time.perf_counter(); render_backward(*args, cfg, grad_hist=grad, **kw); torch.cuda.synchronize()
    bres[flags] = (time.perf_counter() - t0) * 1000
print(json.dumps({'config': cfgname, 'mode': mode, 'cutoff': cutoff, 'ray_cache': cache, 'fwd_ms_by_flags': res, 'bwd_ms_by_flags': bres}))
