"""CPU-only checks of the boundary: the C-ABI library loads, exports every symbol include/nlosgr.h
declares, validates arguments without touching a GPU, and the host-side tables match torch."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "nlosgr.h")).read()
    return sorted(set(re.findall(r"\b(nlosgr_[a-z_]+)\s*\(", src)))


def test_library_exports_header_symbols():
    from nlosgr import _lib
    lib = _lib.load()
    syms = _header_symbols()
    assert syms, "no symbols parsed from header"
    assert sorted(_lib.EXPORTS) == syms
    for s in syms:
        assert hasattr(lib, s), s
    assert lib.nlosgr_abi_version() == _lib.ABI_VERSION


def test_validation_errors_without_gpu():
    """Argument validation runs on the host and reports through nlosgr_last_error."""
    from nlosgr import _lib
    lib = _lib.load()
    g = _lib.Gaussians(10, 25, 5, 0, 1.0, None, None, None, None, None)       # degree 5: unsupported
    geo = _lib.Geometry(1, 4, 4, 8, None, None, None, None, None, None, None, None, None)
    opt = _lib.Options(0, 0.0, 1.0, 1.0, 0, 0)
    rc = lib.nlosgr_render_fwd(g, geo, opt, None, None, None, None)
    assert rc == 3 and b"active_sh_degree" in lib.nlosgr_last_error()
    g = _lib.Gaussians(10, 25, 4, 1, 1.0, None, None, None, None, None)       # degree 4: torch preset only
    rc = lib.nlosgr_render_fwd(g, geo, opt, None, None, None, None)
    assert rc == 3 and b"cuda preset" in lib.nlosgr_last_error()
    g = _lib.Gaussians(10, 16, 4, 0, 1.0, None, None, None, None, None)       # degree 4 needs 25 coefficients
    rc = lib.nlosgr_render_fwd(g, geo, opt, None, None, None, None)
    assert rc == 1 and b"k_feat" in lib.nlosgr_last_error()
    g = _lib.Gaussians(10, 4, 1, 7, 1.0, None, None, None, None, None)        # bad preset
    assert lib.nlosgr_render_fwd(g, geo, opt, None, None, None, None) == 1
    g = _lib.Gaussians(10, 4, 1, 0, 1.0, None, None, None, None, None)        # null param pointers
    assert lib.nlosgr_render_fwd(g, geo, opt, None, None, None, None) == 1
    assert lib.nlosgr_workspace_bytes(g, geo, opt) == 0
    g = _lib.Gaussians(0, 4, 1, 0, 1.0, None, None, None, None, None)         # empty problem is fine
    geo0 = _lib.Geometry(0, 4, 4, 8, None, None, None, None, None, None, None, None, None)
    assert lib.nlosgr_render_fwd(g, geo0, opt, None, None, None, None) == 0


def test_linspace_rows_matches_torch():
    from nlosgr.geometry import linspace_rows
    g = torch.Generator().manual_seed(0)
    lo = torch.rand(50, generator=g) * 2 - 1
    hi = lo + torch.rand(50, generator=g) * 3
    for n in (1, 2, 5, 8, 32, 33):
        got = linspace_rows(lo, hi, n)
        ref = torch.stack([torch.linspace(lo[i].item(), hi[i].item(), n) for i in range(50)])
        assert torch.equal(got, ref), n


def test_batched_tables_match_reference_sampling(golden_case):
    """Batched geometry tables == the reference's per-wall-point spherical_sample_histogram."""
    from nlosgr.geometry import build_geometry
    d = golden_case
    m = d["meta"]
    walls = torch.from_numpy(d["walls"])
    box = torch.from_numpy(d["box"])
    geo = build_geometry(walls, box, m["ns"], m["start"], m["end"], m["c"], m["deltaT"], 0.5, "torch")
    for w in range(m["nwall"]):
        tmin, tmax, pmin, pmax = d["angle_range"][w]
        assert geo.theta[w, 0].item() == np.float32(tmin) and geo.theta[w, -1].item() == np.float32(tmax)
        assert geo.phi[w, 0].item() == np.float32(pmin) and geo.phi[w, -1].item() == np.float32(pmax)
        np.testing.assert_allclose(geo.hscale[w].item(), d["dtheta"][w] * d["dphi"][w] * 0.25, rtol=1e-6)
    ip = torch.from_numpy(d["input_points0"]).view(m["nr"], m["ns"], m["ns"], 5)
    assert torch.equal(geo.theta[0], ip[0, :, 0, 3]) and torch.equal(geo.phi[0], ip[0, 0, :, 4])
    r = ip[:, 0, 0, :3] - walls[0]
    np.testing.assert_allclose(geo.r.numpy(), r.norm(dim=1).numpy(), rtol=1e-5)


def test_geometry_slice_and_wall_grid():
    from nlosgr.geometry import build_geometry, relay_wall_grid, volume_box_point
    walls = relay_wall_grid(4, 6)
    assert walls.shape == (24, 3) and torch.all(walls[:, 1] == 0)
    assert abs(walls[:, 0].mean().item()) < 1e-6 and abs(walls[:, 2].mean().item()) < 1e-6
    geo = build_geometry(walls, volume_box_point((0, 0.5, 0), 0.5), 8, 4, 36, 1.0, 0.04, 0.5, "cuda")
    s = geo.slice(6, 12)
    assert s.nwall == 6 and torch.equal(s.wall, geo.wall[6:12]) and s.nr == 32


def test_dropin_renderers_fail_loudly_without_gpu():
    """The reference's package front (submodules/cuda_renderer/__init__.py) raises when its
    extension is missing; the drop-ins do the same here without a GPU instead of falling back."""
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from nlosgr import cuda_renderer
    assert cuda_renderer.MAX_GAUSSIANS_PER_RAY == 256
    assert cuda_renderer.CUDA_AVAILABLE is False
    with pytest.raises(RuntimeError):
        cuda_renderer.create_renderer(3.0)
    with pytest.raises(RuntimeError):
        cuda_renderer.NLOSGaussianRenderer()


@pytest.mark.parametrize("nwall,nt,np_,nr", [(6, 32, 32, 1024), (3, 7, 5, 40), (2, 32, 32, 2048), (1, 9, 13, 77)])
def test_occl_row_cache_size_matches_library(nwall, nt, np_, nr):
    """render.tile_rows_bytes (the size the Python side checks before enabling the occlusion row
    cache) equals the extra workspace the library plans for it (nlosgr_workspace_bytes with
    ray_cache on minus off; host-only call, no GPU)."""
    from types import SimpleNamespace
    from nlosgr import _lib
    from nlosgr.render import tile_rows_bytes
    lib = _lib.load()
    fake = ctypes.c_void_p(4096)   # validation only checks that the pointers are set
    g = _lib.Gaussians(1000, 16, 3, _lib.PRESET_CUDA, 1.0, fake, fake, fake, fake, fake)
    geo = _lib.Geometry(nwall, nt, np_, nr, *([fake] * 9))
    sizes = []
    for cache in (0, 1):
        opt = _lib.Options(_lib.MODE_OCCL, 3.0, 0.01, 1.0, 0, 0, cache, _lib.SELECT_SUPPORT, 0, 0)
        sizes.append(lib.nlosgr_workspace_bytes(g, geo, opt))
    assert sizes[0] > 0, lib.nlosgr_last_error()
    want = tile_rows_bytes(SimpleNamespace(nwall=nwall, nt=nt, np=np_, nr=nr))
    assert sizes[1] - sizes[0] == (want + 255) // 256 * 256


def test_batch_budgets_restore_the_values_in_effect():
    """batch_budgets restores the budgets that were in effect (nlosgr_get_batch_budgets),
    not the environment's defaults, so nested contexts and direct nlosgr_set_batch_budgets calls survive."""
    from nlosgr import _lib
    lib = _lib.load()

    def get():
        d, h = ctypes.c_double(0.0), ctypes.c_double(0.0)
        lib.nlosgr_get_batch_budgets(ctypes.byref(d), ctypes.byref(h))
        return d.value, h.value

    before = get()
    try:
        lib.nlosgr_set_batch_budgets(77.0, 55.0)
        with _lib.batch_budgets(drho_mb=3.0):
            assert get() == (3.0, 55.0)
            with _lib.batch_budgets(tile_hpart_mb=9.0):
                assert get() == (3.0, 9.0)
            assert get() == (3.0, 55.0)
        assert get() == (77.0, 55.0)
        lib.nlosgr_set_batch_budgets(-5.0, 0.0)      # <= 0 keeps the current values
        assert get() == (77.0, 55.0)
    finally:
        lib.nlosgr_set_batch_budgets(*before)
