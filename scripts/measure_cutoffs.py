"""Work counts and fwd/bwd times of the volume kernels vs the support cutoff (C3 inputs).

    python scripts/measure_cutoffs.py [--config C3] [--cutoffs 3,4,5,5.7,6]
"""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlos-gaussian-renderer_amd")); sys.path.insert(0, ROOT)
import torch
from bench import CONFIGS
from nlosgr import GaussianParams
from nlosgr.model import features_flat
from nlosgr.render import render_forward, render_backward, count_support, use_ray_cache
from nlosgr.volume import Scene, make_config

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--cutoffs", default="3,4,5,5.7,6")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--no-bwd", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda:0")
ng, H, W, T, ns, _ = CONFIGS[a.config]
scene = Scene(H=H, W=W, T=T, ns=ns)
m = GaussianParams.synthetic(ng, 3, preset="cuda", device=dev, seed=0)
geo = scene.geometry(dev, "cuda")
params = [m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
          features_flat(m).detach().contiguous()]
grad = torch.rand(H * W, T, device=dev) * 1e-3
out = []
ref = None
for c in [float(x) for x in a.cutoffs.split(",")]:
    cfg = make_config(m, scene, cutoff=c)
    pairs, rays, evals = count_support(*params, geo, cfg)
    cache = use_ray_cache(cfg, geo, ng)
    tf, tb = [], []
    for _ in range(a.reps):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        o = render_forward(*params, geo, cfg, True, False, ray_cache=cache)
        torch.cuda.synchronize(); t1 = time.perf_counter()
        if not a.no_bwd:
            render_backward(*params, geo, cfg, grad_hist=grad, workspace=o[2] if cache else None, ray_cache=cache)
        torch.cuda.synchronize(); t2 = time.perf_counter()
        tf.append(t1 - t0); tb.append(t2 - t1)
        hist = o[0]
        del o
    if ref is None:
        ref = hist.double()
    rel = ((hist.double() - ref).norm() / ref.norm()).item()
    rec = {"cutoff": c, "pairs": pairs, "rays": rays, "evals": evals, "fwd_ms": 1e3 * min(tf),
           "bwd_ms": 1e3 * min(tb), "rel_vs_first": rel}
    print(json.dumps(rec), flush=True)
    out.append(rec)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", f"cutoffs_{a.config}.json"), "w") as f:
    json.dump(out, f, indent=1)
