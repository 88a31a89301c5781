"""Diagnostic: GPU dense vs culled vs float64 emulation on the cutoff-convergence scene."""
import sys, os, math
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams
from nlosgr.volume import Scene, make_config, render_volume
from oracle import torch_ref as R
dev = torch.device('cuda:0')
scene = Scene(H=8, W=8, T=256, ns=32)
m = GaussianParams.synthetic(2000, 3, preset="cuda", device=dev, seed=1)
geo = scene.geometry(dev, "cuda")
with torch.no_grad():
    dense = render_volume(m, geo, make_config(m, scene, cutoff=0.0)).cpu().double()
    cull = render_volume(m, geo, make_config(m, scene, cutoff=6.0)).cpu().double()
print('gpu cull6 vs dense', ((cull - dense).norm() / dense.norm()).item())
cpu = lambda t: t.detach().cpu().double()
S, Q, mu = cpu(m._scaling), cpu(m._rotation), cpu(m._mu)
st = torch.exp(S) + 1e-8
A = R.quat_to_rotmat_cuda(Q).transpose(1, 2) / st[:, :, None]
sig = torch.sigmoid(cpu(m._opacity))[:, 0]
feats = torch.cat([cpu(m._features_dc).reshape(2000, 1), cpu(m._features_rest).reshape(2000, 15)], 1)
r = cpu(geo.r); att = cpu(geo.att); hs = cpu(geo.hscale)
for p in [0, 27, 63]:
    w = cpu(geo.wall[p]); th = cpu(geo.theta[p]); ph = cpu(geo.phi[p])
    d = torch.stack([torch.sin(th)[:, None] * torch.cos(ph)[None, :], torch.sin(th)[:, None] * torch.sin(ph)[None, :],
                     torch.cos(th)[:, None].expand(32, 32)], -1).reshape(-1, 3)
    q = w[None] - mu
    u0 = torch.einsum('gab,gb->ga', A, q)
    v = torch.einsum('gab,rb->gra', A, d)
    dv = -q; dn = dv * (1 / (dv.norm(dim=1, keepdim=True) + 1e-8))
    wgt = sig * torch.clamp_min(R.eval_sh_cuda(3, feats, dn) + 0.5, 0)
    h = torch.zeros(256)
    for k in range(256):
        z = u0[:, None, :] + r[k] * v
        val = torch.exp(-0.5 * (z * z).sum(-1)) * wgt[:, None] * torch.sin(th).repeat_interleave(32)[None, :]
        h[k] = val.sum()
    h = h * att * hs[p]
    print(p, 'dense vs f64', ((dense[p] - h).norm() / h.norm()).item(), 'cull vs f64', ((cull[p] - h).norm() / h.norm()).item())
    e = (cull[p] - h).abs(); k = int(e.argmax()); print('   worst bin', k, cull[p][k].item(), h[k].item(), dense[p][k].item())
