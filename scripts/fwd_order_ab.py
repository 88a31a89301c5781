"""Forward Gaussian-order A/B (GPU): the C3 forward (default drain) with the Gaussians in their given order
and in slab orders (nlosgr.train.slab_order: slabs x cells x cells, optional size key), medians of --reps;
histograms compared bitwise against the given order (the FX drain is order-independent).

    python scripts/fwd_order_ab.py [--reps 3]"""
import argparse, json, os, statistics, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat
from nlosgr.render import render_forward
from nlosgr.train import slab_order
from nlosgr.volume import Scene, make_config

ap = argparse.ArgumentParser()
ap.add_argument('--reps', type=int, default=3)
ap.add_argument('--mode', default='noocl')
a = ap.parse_args()
dev = torch.device('cuda:0')
scene = Scene(H=128, W=128, T=1024, ns=32)
m = GaussianParams.synthetic(100_000, 3, preset='cuda', device=dev, seed=0)
geo = scene.geometry(dev, 'cuda', a.mode)
cfg = make_config(m, scene, 'cuda', a.mode, cutoff=5.7)
P = [m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), features_flat(m).detach().contiguous()]
size = P[1].max(1).values
orders = {'given': None,
          'slab8x1_size': slab_order(P[0], geo.wall, 8, 1, size=size),
          'slab8x4_size': slab_order(P[0], geo.wall, 8, 4, size=size),
          'slab16x1_size': slab_order(P[0], geo.wall, 16, 1, size=size),
          'size': slab_order(P[0], geo.wall, 1, 1, size=size),
          'slab8x1': slab_order(P[0], geo.wall, 8, 1),
          'slab4x2_size': slab_order(P[0], geo.wall, 4, 2, size=size),
          'slab32x1_size': slab_order(P[0], geo.wall, 32, 1, size=size),
          'slab8x1_sizedesc': slab_order(P[0], geo.wall, 8, 1, size=-size),
          'slab4x1_size': slab_order(P[0], geo.wall, 4, 1, size=size),
          'slab2x1_size': slab_order(P[0], geo.wall, 2, 1, size=size),
          'slab64x1': slab_order(P[0], geo.wall, 64, 1),
          'slab8x2_size': slab_order(P[0], geo.wall, 8, 2, size=size)}
args = {k: (P if o is None else [t[o].contiguous() for t in P]) for k, o in orders.items()}
times = {k: [] for k in orders}
ref = None
same = {}
for rep in range(a.reps + 1):
    for k, pk in args.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h, _ = render_forward(*pk, geo, cfg)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        if rep == 0:
            if ref is None:
                ref = h
            same[k] = bool(torch.equal(h, ref))
            continue
        times[k].append(dt)
print(json.dumps({'mode': a.mode, 'fwd_ms': {k: round(statistics.median(v), 1) for k, v in times.items()},
                  'bitwise_equal_to_given': same}), flush=True)
