"""C2 accuracy (diagnostic): at a few wall points, the culled forward (fixed-point and float drains) and the
dense fp32 evaluation against float64 sums of 250-Gaussian HIP sub-histograms (dense and culled).

    python scripts/fx_accuracy_c2.py [--config C2]
Prints one JSON line."""
import argparse, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat
from nlosgr.render import render_forward
from nlosgr.volume import Scene, make_config

ap = argparse.ArgumentParser()
ap.add_argument('--config', default='C2')
ap.add_argument('--chunk', type=int, default=250)
a = ap.parse_args()
ng, H, T = {'C2': (50_000, 64, 512), 'C3': (100_000, 128, 1024)}[a.config]
dev = torch.device('cuda:0')
scene = Scene(H=H, W=H, T=T, ns=32)
m = GaussianParams.synthetic(ng, 3, preset='cuda', device=dev, seed=0)
P = [m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), features_flat(m).detach().contiguous()]
idx = torch.tensor([0, H * H // 4, H * H // 2 + H // 2, H * H - 1], device=dev)
geo = scene.geometry(dev, 'cuda', 'noocl', walls=scene.walls(dev)[idx].contiguous())
cul = make_config(m, scene, 'cuda', 'noocl', cutoff=5.7)
den = make_config(m, scene, 'cuda', 'noocl', cutoff=0.0)


def fwd(params, cfg, ffx='1'):
    os.environ['NLOSGR_FFX'] = ffx
    try:
        return render_forward(*params, geo, cfg)[0].double()
    finally:
        os.environ.pop('NLOSGR_FFX')


refs = {}
for name, cfg in (('dense', den), ('culled', cul)):
    r = torch.zeros(len(idx), T, dtype=torch.float64, device=dev)
    for g0 in range(0, ng, a.chunk):
        r += fwd([t[g0:g0 + a.chunk].contiguous() for t in P], cfg, '0')
    refs[name] = r
out = {'config': a.config, 'walls': idx.tolist(), 'chunk': a.chunk, 'scale': float(refs['dense'].abs().max()),
       'culled64_vs_dense64': float((refs['culled'] - refs['dense']).abs().max() / refs['dense'].abs().max())}
for name, h in (('fx', fwd(P, cul, '1')), ('float', fwd(P, cul, '0')), ('dense_fp32', fwd(P, den, '0'))):
    for rn, r in refs.items():
        e = h - r
        out[f'{name}_vs_{rn}64'] = {'max_err_of_max': float(e.abs().max() / r.abs().max()),
                                    'mean_signed_rel': float(e.sum() / r.sum())}
print(json.dumps(out), flush=True)
