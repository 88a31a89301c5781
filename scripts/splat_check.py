"""GPU check of the splat kernels: small-scene parity vs the dense oracle, cutoff convergence,
and C3 timings.  python scripts/splat_check.py [--c3]"""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlos-gaussian-renderer_amd")); sys.path.insert(0, ROOT)
import torch
from nlosgr import GaussianParams, features_flat
from nlosgr.geometry import build_geometry, relay_wall_grid, volume_box_point
from nlosgr.render import RenderConfig, render, render_forward, render_backward, count_support
from nlosgr.volume import Scene, make_config, render_volume
from oracle import torch_ref as R

dev = torch.device("cuda:0")
cpu = lambda t: t.detach().cpu()


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max()).item()


def small(preset, cutoff, scale_add=1.2):
    ng, deg, ns, T = 48, 3, 6, 40
    c, deltaT = 1.0, 1.28 / T
    start, end = T // 8, T // 8 + T
    model = GaussianParams.synthetic(ng, deg, preset=preset, device=dev, seed=3)
    if preset == "cuda":
        with torch.no_grad():
            model._scaling.add_(scale_add)
    walls = relay_wall_grid(2, 3, device=dev)
    box = volume_box_point((0.0, 0.5, 0.0), 0.5, dev)
    geo = build_geometry(walls, box, ns, start, end, c, deltaT, 0.5, preset, "noocl")
    cfg = RenderConfig(preset=preset, mode="noocl", sh_degree=deg, cutoff=cutoff, c_deltaT=c * deltaT)
    hist, _ = render(model._mu, model._scaling, model._rotation, model._opacity, features_flat(model), geo, cfg)
    g = torch.Generator().manual_seed(5)
    gout = torch.randn(hist.shape, generator=g)
    (hist * gout.to(dev)).sum().backward()
    params = [cpu(model._mu), cpu(model._scaling), cpu(model._rotation), cpu(model._opacity),
              cpu(model._features_dc), cpu(model._features_rest)]
    P = R.Params(*params, deg)
    ref = R.render_volume(P, cpu(walls), cpu(box), 0.5, ns, start, end, c, deltaT, preset=preset, mode="noocl", mc=None)
    out = {"preset": preset, "cutoff": cutoff, "hist": rel(cpu(hist), ref.detach())}
    (ref * gout).sum().backward()
    for pname, leaf, rleaf in zip(["mu", "scaling", "rotation", "opacity", "dc", "rest"], model.parameters(), P.leaves()):
        out[pname] = rel(cpu(leaf.grad), rleaf.grad)
    return out


for preset, cut in [("cuda", 6.0), ("cuda", 8.0), ("torch", 6.0)]:
    print(json.dumps(small(preset, cut)), flush=True)

scene = Scene(H=8, W=8, T=256, ns=32)
model = GaussianParams.synthetic(2000, 3, preset="cuda", device=dev, seed=1)
geo = scene.geometry(dev, "cuda")
with torch.no_grad():
    dense = render_volume(model, geo, make_config(model, scene, cutoff=0.0))
    errs = {}
    for mc in (3.0, 4.0, 5.0, 5.7, 6.0):
        h = render_volume(model, geo, make_config(model, scene, cutoff=mc))
        errs[mc] = ((h - dense).norm() / dense.norm()).item()
print("cutoff->dense rel L2", json.dumps(errs), flush=True)

if "--c3" in sys.argv:
    from bench import CONFIGS
    ng, H, W, T, ns, _ = CONFIGS["C3"]
    scene = Scene(H=H, W=W, T=T, ns=ns)
    m = GaussianParams.synthetic(ng, 3, preset="cuda", device=dev, seed=0)
    geo = scene.geometry(dev, "cuda")
    params = [m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
              features_flat(m).detach().contiguous()]
    grad = torch.rand(H * W, T, device=dev) * 1e-3
    ref = None
    for cut in [float(x) for x in os.environ.get("CUTS", "6,5.7,5,4,3").split(",")]:
        cfg = make_config(m, scene, cutoff=cut)
        counts = count_support(*params, geo, cfg)
        tf, tb = [], []
        for _ in range(2):
            torch.cuda.synchronize(); t0 = time.perf_counter()
            hist, _ = render_forward(*params, geo, cfg, True, False)
            torch.cuda.synchronize(); t1 = time.perf_counter()
            gr = render_backward(*params, geo, cfg, grad_hist=grad)
            torch.cuda.synchronize(); t2 = time.perf_counter()
            tf.append(t1 - t0); tb.append(t2 - t1)
        if ref is None:
            ref = hist.double(); gref = [g.double() for g in gr]
        print(json.dumps({"cutoff": cut, "counts": counts, "fwd_ms": 1e3 * min(tf), "bwd_ms": 1e3 * min(tb),
                          "hist_rel_vs_first": ((hist.double() - ref).norm() / ref.norm()).item(),
                          "grad_mu_rel_vs_first": ((gr[0].double() - gref[0]).norm() / gref[0].norm()).item(),
                          "finite": bool(torch.isfinite(hist).all() and all(torch.isfinite(g).all() for g in gr))}),
              flush=True)
