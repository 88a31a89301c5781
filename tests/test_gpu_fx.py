"""The fixed-point (FX) forward drain over dynamic range.

The FX drain (csrc/nlosgr_volume.hip, kFxBits) sums every term as an integer count of units 2^-E.  Round 5
took E from the LARGEST amplitude bound of the launch, so a few very bright Gaussians coarsened the unit of
all others and their sub-half-unit tails rounded to zero.  Round 6 takes E from a quantile of the bounds
(the ceil(ng/256)-th brightest) and sends the segments of anything brighter through exact u64 adds into the
global row.  These tests pin:
  * a high-dynamic-range C3 scene (0.1 % of the Gaussians ~4000x brighter than the mean): every sampled
    row within 2e-5 of its own max of the float64 sum of fp32 sub-histograms (the reference sums over all
    Gaussians in fp32: gaussian_model.py:346-364, nlos_helpers.py:228-229), AND the bins the bright ones
    do not reach within 2e-5 of the max of those bins (a stricter test than the row max);
  * the LDS overflow flush (fields past 2^31 moved into the u64 row): a pile of co-located Gaussians that
    forces it, against the CPU oracle;
  * a NaN Gaussian: skipped by the drain and by the unit's quantile, so the others are rendered exactly as
    without it.
The measured errors are printed (pytest -s)."""
from dataclasses import replace

import numpy as np
import pytest
import torch

from conftest import ROOT  # noqa: F401

pytestmark = pytest.mark.gpu

C0 = 0.28209479177387814
CUT = 5.7


def _params(m):
    from nlosgr import features_flat
    return [m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
            features_flat(m).detach().contiguous()]


def _sub(P, idx):
    return [t[idx].contiguous() for t in P]


def _chunk_sum(P, geo, cfg, chunk=250):
    """float64 sum of fp32 float-drain sub-histograms of `chunk` Gaussians each (a few hundred terms per
    bin per sub-histogram: fp32 running sums are accurate to ~1e-7 there)."""
    from nlosgr import _lib
    from nlosgr.render import render_forward
    fcfg = replace(cfg, flags=_lib.FLAG_FLOAT_DRAIN)
    ng = P[0].shape[0]
    ref = torch.zeros(geo.nwall, geo.nr, dtype=torch.float64, device=P[0].device)
    for g0 in range(0, ng, chunk):
        h, _ = render_forward(*[t[g0:g0 + chunk].contiguous() for t in P], geo, fcfg)
        ref += h.double()
    return ref


def _fx(P, geo, cfg, flags=0):
    from nlosgr.render import fx_info, render_forward, workspace_for
    c = replace(cfg, flags=flags)
    ws = workspace_for(*P, geo, c)
    h, _ = render_forward(*P, geo, c, workspace=ws)
    return h.double(), fx_info(*P, geo, c, ws)


def _bright(m, idx, opacity=4.0, rho=200.0):
    """Gaussians idx made bright: sigmoid(opacity) ~ 0.98 and albedo rho (dc only), i.e. sigma*rho ~ 196
    against the synthetic scene's mean ~0.05 (rho ~ U(0, 0.2), opacity ~ N(0, 1))."""
    with torch.no_grad():
        m._opacity[idx] = opacity
        m._features_dc[idx] = (rho - 0.5) / C0
        m._features_rest[idx] = 0.0


def _row_errors(a, ref, ref_bright, ref_dim):
    """(error / row max, error in the bins the bright Gaussians leave alone / the row's DIM content max, mask):
    the second is the precision of the dim Gaussians' own histogram, which a unit set by the bright ones
    would coarsen."""
    row = ((a - ref).abs().max(1).values / ref.abs().max(1).values).cpu().numpy()
    mask = ref_bright < 1e-3 * ref_dim          # bins the bright Gaussians leave (practically) alone
    e = (a - ref).abs()
    dmax = ref_dim.abs().max(1).values
    strict = []
    for i in range(a.shape[0]):
        mk = mask[i]
        strict.append(float(e[i][mk].max() / dmax[i]) if int(mk.sum()) > 0 else 0.0)
    return row, np.array(strict), mask


@pytest.mark.parametrize("mode", ["noocl"])
def test_fx_high_dynamic_range_c3(mode):
    """C3 geometry, 100k Gaussians, every 1000th ~4000x brighter: the FX forward (TrainStep's drain) at
    8 wall points vs the float64 sum of fp32 sub-histograms; per row <= 2e-5 of its max, and
    in the bins the bright Gaussians leave alone <= 2e-5 of the row's dim-Gaussian max (the dim
    Gaussians' own precision).  The round-5 unit (FLAG_FX_MAXUNIT) is
    measured beside it (printed, not asserted)."""
    from nlosgr import GaussianParams, _lib
    from nlosgr.volume import Scene, make_config
    dev = torch.device("cuda:0")
    ng, H, T = 100_000, 128, 1024
    scene = Scene(H=H, W=H, T=T, ns=32)
    m = GaussianParams.synthetic(ng, 3, preset="cuda", device=dev, seed=0)
    bidx = torch.arange(0, ng, 1000, device=dev)
    _bright(m, bidx)
    P = _params(m)
    geo = scene.geometry(dev, "cuda", mode)
    cfg = make_config(m, scene, "cuda", mode, cutoff=CUT)
    widx = torch.linspace(0, H * H - 1, 10, device=dev).long()[1:-1]
    gsel = scene.geometry(dev, "cuda", mode, walls=geo.wall[widx].contiguous())
    dmask = torch.ones(ng, dtype=torch.bool, device=dev)
    dmask[bidx] = False
    ref_dim = _chunk_sum(_sub(P, dmask), gsel, cfg)
    ref_bright = _chunk_sum(_sub(P, bidx), gsel, cfg)
    ref = ref_dim + ref_bright
    a, info = _fx(P, geo, cfg)
    b, info_old = _fx(P, geo, cfg, _lib.FLAG_FX_MAXUNIT)
    a, b = a[widx], b[widx]
    row, strict, mask = _row_errors(a, ref, ref_bright, ref_dim)
    row_o, strict_o, _ = _row_errors(b, ref, ref_bright, ref_dim)
    bshare = (ref_bright.max(1).values / ref.max(1).values).cpu().numpy()
    print(f"\nHDR C3 {mode}: unit E {info[0]} (largest bound's E {info[1]}), bright segments {info[3]}, "
          f"flushes {info[2]}; bright share of row max {np.round(bshare, 3).tolist()}; "
          f"bins left alone per row {mask.sum(1).tolist()}")
    em = ((a - ref).abs() * mask).max(1).values
    print(f"  left-alone bins: ref max {(ref * mask).max(1).values.cpu().numpy()}, dim max "
          f"{ref_dim.max(1).values.cpu().numpy()}, err max {em.cpu().numpy()}")
    print(f"  quantile unit: row err / row max {row.max():.3e}, left-alone bins {strict.max():.3e}, "
          f"mean signed {float(((a - ref).sum() / ref.sum())):.3e}")
    print(f"  round-5 unit (E {info_old[0]}): row err / row max {row_o.max():.3e}, left-alone bins "
          f"{strict_o.max():.3e}, mean signed {float(((b - ref).sum() / ref.sum())):.3e}")
    assert info[3] > 0, "the bright path did not run"
    assert info[0] > info[1], "the unit should be finer than the largest bound's"
    assert row.max() <= 2e-5, row
    assert strict.max() <= 2e-5, strict


@pytest.mark.parametrize("mode", ["noocl", "netf", "binint"])
def test_fx_bright_minority_all_modes(mode):
    """The three FX drains (noocl, netf at c dT <= 1/64, bin-integrated) with 0.25 % of the Gaussians
    ~4000x brighter on a small wall: whole volume vs the float64 sum of fp32 sub-histograms (<= 2e-5 of
    each row's max)."""
    from nlosgr import GaussianParams
    from nlosgr.volume import Scene, make_config
    dev = torch.device("cuda:0")
    ng = 20_000
    scene = Scene(H=6, W=6, T=512, ns=32)
    m = GaussianParams.synthetic(ng, 3, preset="cuda", device=dev, seed=3)
    bidx = torch.arange(7, ng, 400, device=dev)
    _bright(m, bidx)
    P = _params(m)
    geo = scene.geometry(dev, "cuda", mode)
    cfg = make_config(m, scene, "cuda", mode, cutoff=CUT)
    ref = _chunk_sum(P, geo, cfg)
    a, info = _fx(P, geo, cfg)
    row = ((a - ref).abs().max(1).values / ref.abs().max(1).values)
    print(f"\n{mode}: E {info[0]} (max-bound E {info[1]}), bright segments {info[3]}, "
          f"row err / row max {float(row.max()):.3e}")
    assert info[3] > 0
    assert float(row.max()) <= 2e-5


def test_fx_lds_flush_pile_vs_oracle():
    """A pile of 768 co-located, equally bright, wide Gaussians (so none is 'bright': the unit's quantile
    is their common bound) drives a wave's LDS fields past 2^31 units, which moves them into the u64 row
    (the flush branch of the FX drain); the result vs the CPU oracle (cuda preset, 5.7 sigma support)
    <= 2e-5 of the max, and vs the fp32 float drain."""
    from nlosgr import GaussianParams, _lib
    from nlosgr.render import render_forward
    from nlosgr.volume import Scene, make_config
    from oracle import torch_ref as R
    dev = torch.device("cuda:0")
    ng = 768
    scene = Scene(H=2, W=2, T=256, ns=16)
    g = torch.Generator().manual_seed(5)
    mu = torch.tensor(scene.volume_position).float() + 1e-3 * torch.randn(ng, 3, generator=g)
    scaling = torch.full((ng, 3), float(np.log(0.06))) + 0.05 * torch.randn(ng, 3, generator=g)
    rotation = torch.randn(ng, 4, generator=g)
    opacity = torch.full((ng, 1), 4.0)
    fdc = torch.full((ng, 1, 1), (1.0 - 0.5) / C0)
    frest = torch.zeros(ng, 15, 1)
    m = GaussianParams(*(t.float().to(dev).contiguous() for t in (mu, scaling, rotation, opacity, fdc, frest)), 3, 3)
    P = _params(m)
    geo = scene.geometry(dev, "cuda", "noocl")
    cfg = make_config(m, scene, "cuda", "noocl", cutoff=CUT)
    a, info = _fx(P, geo, cfg)
    print(f"\nflush pile: E {info[0]}, flushes {info[2]}, bright segments {info[3]}")
    assert info[2] > 0, "the LDS flush did not run"
    assert info[3] == 0
    cpu = [t.detach().cpu() for t in (m._mu, m._scaling, m._rotation, m._opacity, m._features_dc, m._features_rest)]
    ref = None
    for g0 in range(0, ng, 64):
        Pp = R.Params(*(t[g0:g0 + 64] for t in cpu), 3)
        h = R.render_volume(Pp, scene.walls("cpu"), scene.box("cpu"), scene.volume_position[1], scene.ns,
                            scene.start, scene.end, scene.c, scene.deltaT, preset="cuda", mode="noocl", mc=CUT)
        ref = h.double() if ref is None else ref + h.double()
    err = float((a.cpu() - ref).abs().max() / ref.abs().max())
    hf, _ = render_forward(*P, geo, replace(cfg, flags=_lib.FLAG_FLOAT_DRAIN))
    errf = float((hf.double().cpu() - ref).abs().max() / ref.abs().max())
    print(f"  FX vs oracle {err:.3e} of max (fp32 float drain {errf:.3e})")
    assert err <= 2e-5


def test_fx_nan_gaussian_is_skipped():
    """One NaN opacity among 3000 Gaussians: the FX forward equals the forward without that Gaussian
    (same unit: non-finite bounds are not counted; the drain skips the pair) to 1e-6 of the max (early
    starts of the bank placement depend on the lane order), and stays finite."""
    from nlosgr import GaussianParams
    from nlosgr.volume import Scene, make_config
    dev = torch.device("cuda:0")
    ng = 3000
    scene = Scene(H=4, W=4, T=256, ns=16)
    m = GaussianParams.synthetic(ng, 3, preset="cuda", device=dev, seed=9)
    with torch.no_grad():
        m._opacity[17] = float("nan")
    P = _params(m)
    geo = scene.geometry(dev, "cuda", "noocl")
    cfg = make_config(m, scene, "cuda", "noocl", cutoff=CUT)
    a, info = _fx(P, geo, cfg)
    keep = torch.ones(ng, dtype=torch.bool, device=dev)
    keep[17] = False
    b, info_b = _fx(_sub(P, keep), geo, cfg)
    assert torch.isfinite(a).all()
    assert info[0] == info_b[0], (info, info_b)
    err = float((a - b).abs().max() / b.abs().max())
    print(f"\nNaN Gaussian: E {info[0]}, vs without it {err:.3e} of max")
    assert err <= 1e-6


def test_fx_unit_range_clamp():
    """Bright Gaussians ~1e7x above the quantile's bound: the unit is clamped to 16 binary orders below the
    largest bound's (so the bright launch's u64 sums cannot wrap: a bright term < 2^40 units), and the whole
    volume still matches the float64 sum of fp32 sub-histograms to 2e-5 of each row's max."""
    from nlosgr import GaussianParams
    from nlosgr.volume import Scene, make_config
    dev = torch.device("cuda:0")
    ng = 8000
    scene = Scene(H=4, W=4, T=256, ns=16)
    m = GaussianParams.synthetic(ng, 3, preset="cuda", device=dev, seed=12)
    bidx = torch.arange(5, ng, 800, device=dev)
    _bright(m, bidx, rho=2e6)
    P = _params(m)
    geo = scene.geometry(dev, "cuda", "noocl")
    cfg = make_config(m, scene, "cuda", "noocl", cutoff=CUT)
    ref = _chunk_sum(P, geo, cfg)
    a, info = _fx(P, geo, cfg)
    row = ((a - ref).abs().max(1).values / ref.abs().max(1).values)
    print(f"\nrange clamp: E {info[0]} (max-bound E {info[1]}), bright segments {info[3]}, "
          f"row err / row max {float(row.max()):.3e}")
    assert info[0] == info[1] + 16, info
    assert info[3] > 0
    assert float(row.max()) <= 2e-5
