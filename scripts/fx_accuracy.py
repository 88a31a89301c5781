"""Accuracy of the C3 forward at full Ng (diagnostic): the whole-volume forward with the float claim drain
(NLOSGR_FFX=0) and with the fixed-point drain (default), in the given and in TrainStep's slab order,
against the float64 sum of HIP sub-histograms of 250-Gaussian chunks at a few wall points.

    python scripts/fx_accuracy.py [--walls 4] [--chunk 250]
Prints one JSON line."""
import argparse, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat
from nlosgr.render import render_forward
from nlosgr.train import slab_order
from nlosgr.volume import Scene, make_config

ap = argparse.ArgumentParser()
ap.add_argument('--walls', type=int, default=4)
ap.add_argument('--chunk', type=int, default=250)
ap.add_argument('--cutoff', type=float, default=5.7)
a = ap.parse_args()
dev = torch.device('cuda:0')
ng, H, T = 100_000, 128, 1024
scene = Scene(H=H, W=H, T=T, ns=32)
m = GaussianParams.synthetic(ng, 3, preset='cuda', device=dev, seed=0)
geo = scene.geometry(dev, 'cuda', 'noocl')
cfg = make_config(m, scene, 'cuda', 'noocl', cutoff=a.cutoff)
P = [m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), features_flat(m).detach().contiguous()]
idx = torch.linspace(0, H * H - 1, a.walls + 2, device=dev).long()[1:-1]
gsel = scene.geometry(dev, 'cuda', 'noocl', walls=geo.wall[idx].contiguous())


def fwd(params, g, env):
    old = os.environ.get('NLOSGR_FFX')
    os.environ['NLOSGR_FFX'] = env
    try:
        return render_forward(*params, g, cfg)[0]
    finally:
        if old is None:
            os.environ.pop('NLOSGR_FFX')
        else:
            os.environ['NLOSGR_FFX'] = old


ref = torch.zeros(len(idx), T, dtype=torch.float64, device=dev)
for g0 in range(0, ng, a.chunk):
    sl = slice(g0, min(ng, g0 + a.chunk))
    ref += fwd([t[sl].contiguous() for t in P], gsel, '0').double()
perm = slab_order(P[0], geo.wall, 8, 1, size=P[1].max(1).values)
Pp = [t[perm].contiguous() for t in P]
out = {'config': 'C3', 'cutoff': a.cutoff, 'walls': idx.tolist(), 'chunk': a.chunk, 'vs_float64_chunks': {}}
for name, params, env in (('float_given', P, '0'), ('float_slab', Pp, '0'), ('fx_given', P, '1'), ('fx_slab', Pp, '1')):
    h = fwd(params, geo, env)[idx].double()
    out['vs_float64_chunks'][name] = {'max_err_of_max': float((h - ref).abs().max() / ref.abs().max()),
                                      'rel_l2': float((h - ref).norm() / ref.norm()),
                                      'mean_signed_rel': float(((h - ref).sum() / ref.sum()))}
h0 = fwd(P, geo, '1')
h1 = fwd(Pp, geo, '1')
out['fx_order_independent_bitwise'] = bool(torch.equal(h0, h1))
print(json.dumps(out), flush=True)
