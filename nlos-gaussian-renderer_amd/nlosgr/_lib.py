"""ctypes binding of the C ABI in include/nlosgr.h (libnlosgr.so, built in-tree for gfx950).

There is no CPU fallback: if the library is missing or no GPU is visible, every render call
raises.  torch is imported first so the library binds to the HIP runtime torch loaded.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the ctypes load: shared libamdhip64.so.7)

_HERE = os.path.dirname(os.path.abspath(__file__))
# NLOSGR_LIB overrides the library path (A/B timing of alternative in-tree builds)
LIB_PATH = os.environ.get("NLOSGR_LIB") or os.path.join(_HERE, "libnlosgr.so")

PRESET_TORCH = 0
PRESET_CUDA = 1
MODE_NOOCL = 0
MODE_NETF = 1
MODE_BININT = 2
MODE_OCCL = 3
SELECT_SUPPORT = 0
SELECT_AABB = 1
PRESETS = {"torch": PRESET_TORCH, "cuda": PRESET_CUDA}
MODES = {"noocl": MODE_NOOCL, "netf": MODE_NETF, "binint": MODE_BININT, "occl": MODE_OCCL}
SELECTIONS = {"support": SELECT_SUPPORT, "aabb": SELECT_AABB}

_P = ctypes.c_void_p


class Gaussians(ctypes.Structure):
    _fields_ = [("ng", ctypes.c_int32), ("k_feat", ctypes.c_int32), ("sh_degree", ctypes.c_int32),
                ("preset", ctypes.c_int32), ("scaling_modifier", ctypes.c_float),
                ("mu", _P), ("scaling", _P), ("rotation", _P), ("opacity", _P), ("features", _P)]


class Geometry(ctypes.Structure):
    _fields_ = [("nwall", ctypes.c_int32), ("nt", ctypes.c_int32), ("np", ctypes.c_int32),
                ("nr", ctypes.c_int32), ("wall", _P), ("sin_theta", _P), ("cos_theta", _P),
                ("sin_phi", _P), ("cos_phi", _P), ("grid_lin", _P), ("hscale", _P), ("r", _P),
                ("att", _P)]


class Options(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("cutoff", ctypes.c_float), ("c_deltaT", ctypes.c_float),
                ("ray_scale", ctypes.c_float), ("nsplit", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("ray_cache", ctypes.c_int32), ("selection", ctypes.c_int32), ("g_begin", ctypes.c_int32),
                ("g_end", ctypes.c_int32)]


class Rays(ctypes.Structure):
    _fields_ = [("nrays", ctypes.c_int32), ("nsamp", ctypes.c_int32), ("origins", _P), ("dirs", _P),
                ("t", _P), ("cam", _P)]


class AdamGroup(ctypes.Structure):
    _fields_ = [("param", _P), ("grad", _P), ("exp_avg", _P), ("exp_avg_sq", _P), ("n", ctypes.c_longlong),
                ("lr", ctypes.c_double)]


ADAM_MAX_GROUPS = 8  # NLOSGR_ADAM_MAX_GROUPS
MAX_PER_RAY = 256   # NLOSGR_MAX_PER_RAY
ABI_VERSION = 8     # NLOSGR_ABI_VERSION

# nlosgr_options.flags variant selection (NLOSGR_FLAG_*; A/B timing and parity cross-checks, 0 in production)
FLAG_FLOAT_DRAIN = 0x100   # forward: fp32 claim drain instead of the fixed-point drain
FLAG_MASKED_FWD = 0x200    # forward: masked drains at every cutoff (no TAIL)
FLAG_MASKED_BWD = 0x400    # backward: masked drains at every cutoff (no TAIL)
FLAG_LANE_DENSE = 0x800    # dense no-occlusion histogram through the lane-serial drain
FLAG_BWD_SHARED = 0x1000   # backward: shared-row layout
FLAG_BWD_PERWAVE = 0x2000  # backward: per-wave row layout
FLAG_FX_MAXUNIT = 0x4000   # FX drain unit from the largest bound (round-5 rule; diagnostics)
FLAG_TILE_NOBIN = 0x8000   # ray-tile engine: in-kernel cull instead of the tile bins (A/B)

# every symbol include/nlosgr.h declares (tests check the exports against this list)
EXPORTS = ["nlosgr_workspace_bytes", "nlosgr_render_fwd", "nlosgr_render_bwd", "nlosgr_count_support", "nlosgr_fx_info",
           "nlosgr_bboxes", "nlosgr_rays_workspace_bytes", "nlosgr_filter_rays", "nlosgr_rays_fwd",
           "nlosgr_rays_bwd", "nlosgr_rays_analytic", "nlosgr_mse_workspace_bytes", "nlosgr_mse", "nlosgr_adam",
           "nlosgr_carve_votes", "nlosgr_set_batch_budgets", "nlosgr_get_batch_budgets", "nlosgr_last_error", "nlosgr_abi_version"]

_lib = None
_load_error = None


def load():
    """Load (once) and return the library; raises if it is missing."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"nlosgr: HIP library not built: {LIB_PATH} "
                           "(run python nlos-gaussian-renderer_amd/build.py)")
    lib = ctypes.CDLL(LIB_PATH)
    PG, PGEO, POPT = ctypes.POINTER(Gaussians), ctypes.POINTER(Geometry), ctypes.POINTER(Options)
    lib.nlosgr_workspace_bytes.argtypes = [PG, PGEO, POPT]
    lib.nlosgr_workspace_bytes.restype = ctypes.c_size_t
    lib.nlosgr_render_fwd.argtypes = [PG, PGEO, POPT, _P, _P, _P, _P]
    lib.nlosgr_render_fwd.restype = ctypes.c_int
    lib.nlosgr_render_bwd.argtypes = [PG, PGEO, POPT, _P, _P, _P, _P, _P, _P, _P, _P, _P]
    lib.nlosgr_render_bwd.restype = ctypes.c_int
    lib.nlosgr_count_support.argtypes = [PG, PGEO, POPT, _P, _P, _P]
    lib.nlosgr_count_support.restype = ctypes.c_int
    lib.nlosgr_fx_info.argtypes = [PG, PGEO, POPT, _P, _P, _P]
    lib.nlosgr_fx_info.restype = ctypes.c_int
    PR = ctypes.POINTER(Rays)
    lib.nlosgr_rays_workspace_bytes.argtypes = [PG, PR]
    lib.nlosgr_rays_workspace_bytes.restype = ctypes.c_size_t
    lib.nlosgr_filter_rays.argtypes = [PG, PR, _P, _P, _P]
    lib.nlosgr_filter_rays.restype = ctypes.c_int
    lib.nlosgr_rays_fwd.argtypes = [PG, PR, _P, ctypes.c_float, ctypes.c_int32, _P, _P, _P, _P, _P]
    lib.nlosgr_rays_fwd.restype = ctypes.c_int
    lib.nlosgr_rays_bwd.argtypes = [PG, PR, _P, ctypes.c_float, ctypes.c_int32, _P, _P, _P, _P, _P, _P, _P,
                                    _P, _P, _P]
    lib.nlosgr_rays_bwd.restype = ctypes.c_int
    lib.nlosgr_rays_analytic.argtypes = [PG, PR, _P, ctypes.c_float, ctypes.c_float, ctypes.c_float, _P, _P]
    lib.nlosgr_rays_analytic.restype = ctypes.c_int
    lib.nlosgr_mse_workspace_bytes.argtypes = []
    lib.nlosgr_mse_workspace_bytes.restype = ctypes.c_size_t
    lib.nlosgr_mse.argtypes = [_P, _P, ctypes.c_float, ctypes.c_longlong, ctypes.c_float, _P, _P, _P, _P]
    lib.nlosgr_mse.restype = ctypes.c_int
    lib.nlosgr_adam.argtypes = [ctypes.POINTER(AdamGroup), ctypes.c_int32, ctypes.c_longlong, ctypes.c_double,
                                ctypes.c_double, ctypes.c_double, _P]
    lib.nlosgr_adam.restype = ctypes.c_int
    lib.nlosgr_carve_votes.argtypes = [_P, ctypes.c_longlong, _P, _P, ctypes.c_int32, _P, _P]
    lib.nlosgr_carve_votes.restype = ctypes.c_int
    lib.nlosgr_bboxes.argtypes = [PG, ctypes.c_float, _P, _P]
    lib.nlosgr_bboxes.restype = ctypes.c_int
    lib.nlosgr_set_batch_budgets.argtypes = [ctypes.c_double, ctypes.c_double]
    lib.nlosgr_set_batch_budgets.restype = None
    lib.nlosgr_get_batch_budgets.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    lib.nlosgr_get_batch_budgets.restype = None
    lib.nlosgr_last_error.argtypes = []
    lib.nlosgr_last_error.restype = ctypes.c_char_p
    lib.nlosgr_abi_version.argtypes = []
    lib.nlosgr_abi_version.restype = ctypes.c_int
    if lib.nlosgr_abi_version() != ABI_VERSION:
        raise RuntimeError("nlosgr: ABI version mismatch")
    _lib = lib
    return lib


def available():
    """True when the library loads and a GPU is visible (CUDA_AVAILABLE of the reference API)."""
    try:
        load()
    except Exception:
        return False
    return torch.cuda.is_available()


def check(rc):
    if rc != 0:
        msg = load().nlosgr_last_error().decode(errors="replace")
        raise RuntimeError(f"nlosgr error {rc}: {msg}")


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def stream_handle(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class batch_budgets:
    """Context manager: nlosgr_set_batch_budgets(drho_mb, tile_hpart_mb) inside, the previous values
    restored on exit (None keeps a value).  The budgets shape the workspace layout, so no workspace
    sized under other values may be used inside (tests force wall-point batches this way)."""

    def __init__(self, drho_mb=None, tile_hpart_mb=None):
        self.new = (drho_mb, tile_hpart_mb)

    def __enter__(self):
        d, h = ctypes.c_double(0.0), ctypes.c_double(0.0)
        load().nlosgr_get_batch_budgets(ctypes.byref(d), ctypes.byref(h))   # the values in effect
        self.old = (d.value, h.value)
        load().nlosgr_set_batch_budgets(*(float(v) if v is not None else -1.0 for v in self.new))
        return self

    def __exit__(self, *exc):
        load().nlosgr_set_batch_budgets(*self.old)
        return False
