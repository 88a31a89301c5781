"""Generate golden vectors by running the REFERENCE's own PyTorch numerical path (path T).

Runs ONLY in the build container, where /root/reference is mounted read-only.  It imports
the reference with the non-invasive shims recorded in SURVEY.md Appendix B and writes small
fp32 .npz fixtures into tests/golden/.  Nothing under /root/reference is copied: each fixture
holds inputs (raw Gaussian parameters, wall points, geometry scalars) and the reference's
outputs for them.  Tests compare the oracle (oracle/torch_ref.py) and the HIP kernels
against these files; the GPU box never sees the reference.

Reference call chain exercised (file:line under /root/reference):
  nlos_helpers.compute_loss                      nlos_helpers.py:280-346
    -> spherical_sample_histogram                nlos_helpers.py:124-188
    -> gaussian_transient_rendering              nlos_helpers.py:192-232
       -> GaussianModel.estimate_rho_w_no_occlusion  gaussian_model/gaussian_model.py:346-364
       -> GaussianModel.estimate_rho_w ('netf')      gaussian_model/gaussian_model.py:297-325
  loss.backward()  -> grads of the six raw parameters
  unit fixtures: sh_utils.eval_sh :57-112, gaussian_utils.build_rotation :189-210,
                 GaussianModel.estimate_gaussian_pdf :253-294

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import os
import sys
import types
import tempfile
import json

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def import_reference():
    for n in ["open3d", "trimesh", "skimage", "skimage.measure", "cv2"]:  # off-path deps, absent
        sys.modules.setdefault(n, types.ModuleType(n))
    sys.modules["skimage.measure"].marching_cubes = None
    sys.path.insert(0, REF)
    import gaussian_model.gaussian_utils as gu
    gu.inverse_opacity_activation = gu.inverse_sigmoid  # name imported at gaussian_model.py:4, never defined
    from gaussian_model.gaussian_model import GaussianModel
    import gaussian_model.sh_utils as shu
    import nlos_helpers as H
    from configs.default import Config
    return gu, shu, GaussianModel, H, Config


def synth_params(ng, deg, seed):
    """Synthetic raw parameters (SURVEY §8d recipe, torch preset)."""
    g = torch.Generator().manual_seed(seed)
    center = torch.tensor([0.0, 0.5, 0.0])
    size = 0.5
    pmin = center - size / 2
    pmax = center + size / 2
    lo = pmin + (pmin * 0.1).abs()
    hi = pmax - (pmax * 0.1).abs()
    mu = torch.rand(ng, 3, generator=g) * (hi - lo) + lo
    K = (deg + 1) ** 2
    scaling = torch.randn(ng, 3, generator=g) * 0.7 - 1.0      # exp(exp(.)) -> anisotropic, >= 1
    rotation = torch.randn(ng, 4, generator=g)
    opacity = torch.randn(ng, 1, generator=g)
    rho = torch.rand(ng, 1, generator=g) * 0.2
    fdc = ((rho - 0.5) / 0.28209479177387814).reshape(ng, 1, 1)
    frest = 0.05 * torch.randn(ng, K - 1, 1, generator=g)
    return dict(mu=mu, scaling=scaling, rotation=rotation, opacity=opacity,
                features_dc=fdc, features_rest=frest)


def wall_points(nw, seed):
    g = torch.Generator().manual_seed(seed)
    xz = torch.rand(nw, 2, generator=g) - 0.5
    return torch.stack([xz[:, 0], torch.zeros(nw), xz[:, 1]], dim=1)  # plane y = 0


def run_case(name, ng, ns, nr, deg, nwall, occlusion, seed, out):
    gu, shu, GaussianModel, H, Config = import_reference()
    args = Config().to_namespace()
    args.num_sampling_points = ns
    args.start = max(1, nr // 8)
    args.end = args.start + nr
    args.sh_degree = deg
    args.occlusion = occlusion
    args.rendering_type = "netf"
    args.save_fig = False
    args.scaling_modifier = 1.0
    args.gt_times = 100

    c = 1.0
    deltaT = 1.28 / nr
    volume_position = torch.tensor([0.0, 0.5, 0.0])
    volume_size = 0.5
    box = torch.tensor(H.volume_box_point(volume_position.numpy(), volume_size), dtype=torch.float)
    walls = wall_points(nwall, seed + 1)
    gtar = torch.Generator().manual_seed(seed + 2)
    L = args.end + 4
    nlos_data = torch.rand(L, 1, nwall, generator=gtar) * 1e-3     # [L, M=1, N=nwall]
    data_kwargs = {
        "nlos_data": nlos_data,
        "camera_grid_positions": walls.t().contiguous(),            # [3, M*N]
        "volume_position": volume_position,
        "volume_size": volume_size,
        "volume_box_point": box,
        "deltaT": deltaT,
        "c": c,
        "pmin": torch.zeros(5),
        "pmax": torch.zeros(5),
    }
    p = synth_params(ng, deg, seed)
    model = GaussianModel(args, torch.device("cpu"))
    model._mu = torch.nn.Parameter(p["mu"].clone())
    model._scaling = torch.nn.Parameter(p["scaling"].clone())
    model._rotation = torch.nn.Parameter(p["rotation"].clone())
    model._opacity = torch.nn.Parameter(p["opacity"].clone())
    model._features_dc = torch.nn.Parameter(p["features_dc"].clone())
    model._features_rest = torch.nn.Parameter(p["features_rest"].clone())
    model.active_sh_degree = deg

    crit = torch.nn.MSELoss(reduction="mean")
    rec = {k: v.numpy() for k, v in p.items()}
    rec.update(walls=walls.numpy(), box=box.numpy(), nlos_data=nlos_data.numpy(),
               volume_position=volume_position.numpy())
    meta = dict(name=name, ng=ng, ns=ns, nr=nr, deg=deg, nwall=nwall, occlusion=occlusion,
                start=args.start, end=args.end, c=c, deltaT=deltaT, gt_times=args.gt_times,
                volume_size=volume_size, rendering_type=args.rendering_type,
                torch_version=torch.__version__)
    total = 0.0
    hists, results, losses, eqs, I1s, I2s, dths, dphs, tmm = [], [], [], [], [], [], [], [], []
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)   # compute_loss writes ./loss_compare.mat on every call (nlos_helpers.py:343-344)
        try:
            for w in range(nwall):
                optim_kwargs = {"m": 0, "N": nwall, "n": w, "criterion": crit, "current_iter": 1}
                cam = data_kwargs["camera_grid_positions"][:, w]
                with torch.no_grad():
                    ip, I1, I2, num_r, dth, dph, tmin, tmax, pmin_, pmax_ = \
                        H.spherical_sample_histogram(args, data_kwargs, cam)
                result, hist = H.gaussian_transient_rendering(args, model, data_kwargs, ip, cam,
                                                              I1, I2, num_r, dth, dph)
                loss, eq = H.compute_loss(args, model, data_kwargs, optim_kwargs, torch.device("cpu"))
                total = total + loss
                hists.append(hist.detach().numpy())
                results.append(result.detach().numpy())
                losses.append(float(loss))
                eqs.append(float(eq))
                I1s.append(I1); I2s.append(I2); dths.append(dth); dphs.append(dph)
                tmm.append([tmin, tmax, pmin_, pmax_])
                if w == 0:
                    rec["input_points0"] = ip.numpy()
        finally:
            os.chdir(cwd)
    total.backward()
    rec.update(hist=np.stack(hists), result=np.stack(results), loss=np.array(losses),
               equal_loss=np.array(eqs), I1=np.array(I1s), I2=np.array(I2s),
               dtheta=np.array(dths), dphi=np.array(dphs), angle_range=np.array(tmm),
               grad_mu=model._mu.grad.numpy(), grad_scaling=model._scaling.grad.numpy(),
               grad_rotation=model._rotation.grad.numpy(), grad_opacity=model._opacity.grad.numpy(),
               grad_features_dc=model._features_dc.grad.numpy(),
               grad_features_rest=model._features_rest.grad.numpy())
    rec["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(out, f"{name}.npz"), **rec)
    print(name, "hist max", np.abs(rec["hist"]).max(), "loss", losses)


CASES = {
    "noocl_g32_s4_r16_d4": dict(ng=32, ns=4, nr=16, deg=4, nwall=2, occlusion=False, seed=70),
    "netf_g32_s4_r16_d4": dict(ng=32, ns=4, nr=16, deg=4, nwall=1, occlusion=True, seed=80),
}


def run_units(out):
    gu, shu, GaussianModel, H, Config = import_reference()
    g = torch.Generator().manual_seed(7)
    rec = {}
    dirs = torch.nn.functional.normalize(torch.randn(64, 3, generator=g), dim=1)
    for deg in range(5):
        K = (deg + 1) ** 2
        sh = torch.randn(64, 1, K, generator=g)
        rec[f"sh{deg}_coef"] = sh.numpy()
        rec[f"sh{deg}_out"] = shu.eval_sh(deg, sh, dirs).numpy()
    rec["sh_dirs"] = dirs.numpy()
    q = torch.randn(32, 4, generator=g)
    rec["rot_q"] = q.numpy()
    rec["rot_R"] = gu.build_rotation(q).numpy()

    args = Config().to_namespace()
    model = GaussianModel(args, torch.device("cpu"))
    ng = 8
    model._mu = torch.rand(ng, 3, generator=g)
    model._scaling = torch.randn(ng, 3, generator=g) * 0.5 - 1.0
    model._rotation = torch.randn(ng, 4, generator=g)
    x = torch.rand(50, 3, generator=g) * 2 - 0.5
    rec.update(pdf_mu=model._mu.numpy(), pdf_scaling=model._scaling.numpy(),
               pdf_rotation=model._rotation.numpy(), pdf_x=x.numpy(),
               pdf_out=model.estimate_gaussian_pdf(x, 1.0).numpy(),
               pdf_out_mod=model.estimate_gaussian_pdf(x, 0.7).numpy())
    np.savez_compressed(os.path.join(out, "units.npz"), **rec)
    print("units written")


if __name__ == "__main__":
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    out = HERE
    only = sys.argv[1:]   # optional case names: regenerate just those
    if only:
        for name in only:
            kw = dict(CASES[name])
            run_case(name, out=out, **kw)
        sys.exit(0)
    run_units(out)
    run_case("noocl_g16_s4_r16_d0", ng=16, ns=4, nr=16, deg=0, nwall=1, occlusion=False, seed=10, out=out)
    run_case("noocl_g64_s8_r32_d3", ng=64, ns=8, nr=32, deg=3, nwall=2, occlusion=False, seed=20, out=out)
    run_case("netf_g64_s4_r16_d3", ng=64, ns=4, nr=16, deg=3, nwall=2, occlusion=True, seed=30, out=out)
    run_case("noocl_g256_s8_r64_d3", ng=256, ns=8, nr=64, deg=3, nwall=1, occlusion=False, seed=40, out=out)
    run_case("netf_g32_s8_r64_d1", ng=32, ns=8, nr=64, deg=1, nwall=1, occlusion=True, seed=50, out=out)
    run_case("noocl_g16_s5_r24_d2", ng=16, ns=5, nr=24, deg=2, nwall=3, occlusion=False, seed=60, out=out)
    # SH degree 4 (sh_utils.py:102-112; torch preset only)
    run_case("noocl_g32_s4_r16_d4", ng=32, ns=4, nr=16, deg=4, nwall=2, occlusion=False, seed=70, out=out)
    run_case("netf_g32_s4_r16_d4", ng=32, ns=4, nr=16, deg=4, nwall=1, occlusion=True, seed=80, out=out)
