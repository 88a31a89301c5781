"""One C3-size forward + backward of the ray-tile engine (occlusion / AABB selection), timed with
HIP events; with a diagnostic build (NLOSGR_TILES_DIAG_BUILD=1, NLOSGR_TILES_DIAG=1) the engine also
prints per-phase slot-cycles.  Diagnostic only.
    python scripts/occl_phase.py [--selection aabb|support] [--cutoff 5.7] [--mode occl|noocl] [--hw 128]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlos-gaussian-renderer_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--selection", default="aabb")
    ap.add_argument("--cutoff", type=float, default=5.7)
    ap.add_argument("--mode", default="occl")
    ap.add_argument("--hw", type=int, default=128)
    ap.add_argument("--ng", type=int, default=100_000)
    a = ap.parse_args()
    from nlosgr import GaussianParams, features_flat
    from nlosgr.render import render_backward, render_forward
    from nlosgr.volume import Scene, make_config
    dev = torch.device("cuda:0")
    scene = Scene(H=a.hw, W=a.hw, T=1024, ns=32)
    m = GaussianParams.synthetic(a.ng, 3, preset="cuda", device=dev, seed=0)
    geo = scene.geometry(dev, "cuda", a.mode)
    cfg = make_config(m, scene, "cuda", a.mode, cutoff=a.cutoff, selection=a.selection)
    args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
            features_flat(m).detach().contiguous())
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record()
    hist, _ = render_forward(*args, geo, cfg)
    ev[1].record()
    render_backward(*args, geo, cfg, grad_hist=torch.randn_like(hist) * 1e-3)
    ev[2].record()
    torch.cuda.synchronize()
    print(json.dumps({"selection": a.selection, "mode": a.mode, "cutoff": a.cutoff, "hw": a.hw,
                      "fwd_ms": ev[0].elapsed_time(ev[1]), "bwd_ms": ev[1].elapsed_time(ev[2])}), flush=True)


if __name__ == "__main__":
    main()
