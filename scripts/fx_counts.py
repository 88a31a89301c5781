"""Bank-pair occupancy of the FX forward drain at C3 (debug build -DNLOSGR_FXCOUNT, selected by NLOSGR_LIB):
per drain round the active lanes, sum over the 4 16-lane groups of the largest number of lanes on one bank
pair (the ds_add_u64's LDS-array cycles; 4 = conflict-free), distinct bank pairs in the wave and the
wave's largest residue count.     python scripts/fx_counts.py [order: given|train]"""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'nlos-gaussian-renderer_amd')); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat, _lib
from nlosgr.volume import Scene, make_config
from nlosgr.render import render_forward
from nlosgr.train import slab_order, wall_centroid
order = sys.argv[1] if len(sys.argv) > 1 else 'train'
dev = torch.device('cuda:0')
scene = Scene(H=128, W=128, T=1024, ns=32)
m = GaussianParams.synthetic(100_000, 3, preset='cuda', device=dev, seed=0)
geo = scene.geometry(dev, 'cuda')
args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(), features_flat(m).detach())
if order == 'train':
    perm = slab_order(args[0], None, 8, 1, size=args[1].max(1).values, centroid=wall_centroid(geo.wall))
    args = tuple(t[perm].contiguous() for t in args)
cfg = make_config(m, scene, 'cuda', cutoff=5.7)
lib = _lib.load()
f = lib.nlosgr_debug_fx_counts
f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 8)()
torch.cuda.synchronize(); f(buf)
render_forward(*args, geo, cfg)
torch.cuda.synchronize(); f(buf)
c = list(buf)
r = max(c[0], 1)
print(json.dumps({"lib": os.environ.get("NLOSGR_LIB", "in-tree"), "order": order, "rounds": c[0],
                  "active_per_round": c[1] / r, "sum_group_max_per_round": c[2] / r,
                  "distinct_residues_per_round": c[3] / r, "wave_max_residue_count_per_round": c[4] / r}))
