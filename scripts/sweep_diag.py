"""Diagnostic (GPU): sweep forward vs lane-serial TAIL drain vs dense on a C3-like geometry; for each
library in NLOSGR_DIAG_LIBS (comma list, '' = default build) prints rel-L2 / max-rel of every pair
and where the largest sweep-vs-lane-serial differences sit.  Run each library in its own process."""
import os
import sys
from dataclasses import replace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlos-gaussian-renderer_amd"))
sys.path.insert(0, ROOT)


def main():
    from nlosgr import GaussianParams, features_flat
    from nlosgr.render import render_forward
    from nlosgr.volume import Scene, make_config
    preset = os.environ.get("DIAG_PRESET", "cuda")
    ng = int(os.environ.get("DIAG_NG", "6000"))
    dev = torch.device("cuda:0")
    scene = Scene(H=3, W=3, T=1024, ns=32)
    m = GaussianParams.synthetic(ng, 3, preset=preset, device=dev, seed=21)
    geo = scene.geometry(dev, preset)
    args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
            features_flat(m).detach().contiguous(), geo)
    cfg = make_config(m, scene, preset, cutoff=5.7)
    os.environ.pop("NLOSGR_FSWEEP", None)
    sw, _ = render_forward(*args, cfg)
    os.environ["NLOSGR_FSWEEP"] = "0"
    ls, _ = render_forward(*args, cfg)
    os.environ.pop("NLOSGR_FSWEEP", None)
    dn, _ = render_forward(*args, replace(cfg, cutoff=0.0))
    hi, _ = render_forward(*args, replace(cfg, cutoff=8.0))
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()
    mx = lambda a, b: ((a - b).abs().max() / b.abs().max()).item()
    print(f"lib {os.environ.get('NLOSGR_LIB', 'default')} preset {preset} ng {ng}")
    for n, a, b in (("sweep-dense", sw, dn), ("ls-dense", ls, dn), ("sweep-ls", sw, ls), ("ls8-dense", hi, dn)):
        print(f"  {n:12s} relL2 {rel(a, b):.3e} maxrel {mx(a, b):.3e}")
    d = (sw - ls).abs()
    v, i = d.flatten().topk(8)
    for vv, ii in zip(v.tolist(), i.tolist()):
        p, k = divmod(ii, scene.T)
        print(f"  p {p} bin {k}: sweep {sw[p, k].item():.6e} ls {ls[p, k].item():.6e} dense {dn[p, k].item():.6e}")
    print("  sums", sw.sum().item(), ls.sum().item(), dn.sum().item())


if __name__ == "__main__":
    main()
