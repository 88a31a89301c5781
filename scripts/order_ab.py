"""A/B (GPU): the C3 forward/backward with the Gaussians in their given order vs sorted along a
space-filling (Morton) curve of their means, same Gaussians; medians of --reps, rel-L2 of the
histograms.   python scripts/order_ab.py [--cutoff 5.7] [--reps 3] [--bits 10]"""
import argparse, json, os, statistics, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat
from nlosgr.volume import Scene, make_config
from nlosgr.render import render_backward, render_forward

ap = argparse.ArgumentParser()
ap.add_argument('--cutoff', type=float, default=5.7)
ap.add_argument('--reps', type=int, default=3)
ap.add_argument('--keys', default='morton,y,smax,ydist')
a = ap.parse_args()
dev = torch.device('cuda:0')
scene = Scene(H=128, W=128, T=1024, ns=32)
m = GaussianParams.synthetic(100_000, 3, preset='cuda', device=dev, seed=0)
geo = scene.geometry(dev, 'cuda')
cfg = make_config(m, scene, 'cuda', cutoff=a.cutoff)
base = [m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), features_flat(m).detach()]


def morton(mu, bits=10):
    lo, hi = mu.min(0).values, mu.max(0).values
    q = ((mu - lo) / (hi - lo + 1e-9) * (2 ** bits - 1)).long()
    code = torch.zeros(mu.shape[0], dtype=torch.long, device=mu.device)
    for b in range(bits):
        for d in range(3):
            code |= ((q[:, d] >> b) & 1) << (3 * b + d)
    return code


KEYS = {'morton': lambda: morton(base[0]), 'morton6': lambda: morton(base[0], 6), 'y': lambda: base[0][:, 1],
        'smax': lambda: base[1].max(1).values,
        # distance from the wall's centre (0, 0, 0) -> chunk box sizes alike, start bins still spread
        'ydist': lambda: base[0].norm(dim=1),
        'xzy': lambda: (base[0][:, 1] * 16).floor() * 64 + (base[0][:, 0] * 8).floor() * 8 + (base[0][:, 2] * 8).floor()}
variants = [('given', base)]
for kname in a.keys.split(','):
    perm = torch.argsort(KEYS[kname]())
    variants.append((kname, [t[perm].contiguous() for t in base]))
g = torch.randn(scene.H * scene.W, scene.T, device=dev, generator=torch.Generator(device=dev).manual_seed(0)) * 1e-3
res = {}
hists = {}
for rep in range(a.reps + 1):
    for name, p in variants:
        torch.cuda.synchronize(); t0 = time.perf_counter()
        h, _ = render_forward(*p, geo, cfg)
        torch.cuda.synchronize(); t1 = time.perf_counter()
        render_backward(*p, geo, cfg, grad_hist=g)
        torch.cuda.synchronize(); t2 = time.perf_counter()
        if rep:
            res.setdefault(name, []).append(((t1 - t0) * 1e3, (t2 - t1) * 1e3))
        hists[name] = h
out = {n: {'fwd_ms': statistics.median(x[0] for x in v), 'bwd_ms': statistics.median(x[1] for x in v)} for n, v in res.items()}
out['rel_l2'] = {n: ((hists[n] - hists['given']).norm() / hists['given'].norm()).item() for n, _ in variants}
print(json.dumps(out))
