"""Forward drain utilisation at C3 (diagnostic flags 8 of count_support): wave drain rounds,
active lanes and claim winners per round, against the in-support samples."""
import dataclasses, os, sys, json  # needs a -D NLOSGR_DIAG=1 build (NLOSGR_LIB=...)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat
from nlosgr.volume import Scene, make_config
from nlosgr.render import count_support, render_backward, render_forward
cfgname = sys.argv[1] if len(sys.argv) > 1 else 'C3'
ng, H, T = {'C3': (100_000, 128, 1024), 'S1': (20_000, 32, 512)}[cfgname]
dev = torch.device('cuda:0')
scene = Scene(H=H, W=H, T=T, ns=32)
m = GaussianParams.synthetic(ng, 3, preset="cuda", device=dev, seed=0)
geo = scene.geometry(dev, "cuda")
args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), features_flat(m).detach(), geo)
base = make_config(m, scene, cutoff=3.0)
pairs, segs, samples = count_support(*args, base)
rounds, act, win = count_support(*args, dataclasses.replace(base, flags=8))
_, _, cells = count_support(*args, dataclasses.replace(base, flags=16))
print(json.dumps({"pairs": pairs, "segments": segs, "samples": samples, "rounds": rounds,
                  "active_per_round": act / rounds, "winners_per_round": win / rounds,
                  "useful_bins_per_round": samples / rounds, "bins_per_segment": samples / segs,
                  "candidate_cells": cells, "cells_per_pair": cells / pairs, "rays_per_pair": segs / pairs}))

hist, _, ws = render_forward(*args, base, ray_cache=True)
grad = torch.randn_like(hist) * 1e-3
render_backward(*args, dataclasses.replace(base, flags=8), grad_hist=grad, workspace=ws, ray_cache=True)
torch.cuda.synchronize()
d = ws[-256:].view(torch.int64)[:5].tolist()
print(json.dumps({"bwd_drain_rounds": d[0], "bwd_active_per_round": d[1] / max(1, d[0]),
                  "handoff_rounds": d[2], "pending_per_handoff": d[3] / max(1, d[2]),
                  "winners_per_handoff": d[4] / max(1, d[2]), "rays": segs}))
