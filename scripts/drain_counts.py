"""Forward drain utilisation at C3 from a debug build (-DNLOSGR_FCOUNT, selected by NLOSGR_LIB):
count_support then returns (wave rounds, active lanes summed over rounds, claim winners summed)."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat
from nlosgr.volume import Scene, make_config
from nlosgr.render import count_support
cut = float(sys.argv[1]) if len(sys.argv) > 1 else 5.7
dev = torch.device('cuda:0')
scene = Scene(H=128, W=128, T=1024, ns=32)
m = GaussianParams.synthetic(100_000, 3, preset='cuda', device=dev, seed=0)
geo = scene.geometry(dev, 'cuda')
args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), features_flat(m).detach(), geo)
r, a, w = count_support(*args, make_config(m, scene, 'cuda', cutoff=cut))
print(json.dumps({"lib": os.environ.get("NLOSGR_LIB"), "cutoff": cut, "rounds": r, "active_per_round": a / r,
                  "winners_per_round": w / r / 64}))
