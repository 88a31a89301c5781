"""Captured-data path around the renderer: the Zaragoza transient format, the
reference's data_kwargs / data_shuffle, and the whole-volume targets and geometry the fused
training step consumes.

The reference imports `load_zaragoza256_data` from `data.data_loader` (main.py:17, :93), a module
that is not in the repository. `load_zaragoza` restates the published loader of the
Zaragoza NLOS captures that call site expects (NeTF's `load_zaragoza256_data`): a MATLAB v5 file
with `data` [T, H, W] (optionally with leading singleton axes), `cameraPosition` [3],
`cameraGridSize` [2], `cameraGridPositions` [3, H*W], `cameraGridPoints` [2],
`hiddenVolumePosition` [3], `hiddenVolumeSize`, `deltaT`, `c`; it returns the same 9-tuple in the
same order (main.py:93). No captured file ships with the reference, so the format is pinned only
by that call site (parity unpinned; tests/test_data_cpu.py round-trips a synthetic file).
MATLAB v7.3 (HDF5) files need h5py, which this image lacks: they raise with that message.
"""
import numpy as np
import torch

from .geometry import build_geometry, volume_box_point

ZARAGOZA_KEYS = ("data", "cameraPosition", "cameraGridSize", "cameraGridPositions", "cameraGridPoints",
                 "hiddenVolumePosition", "hiddenVolumeSize", "deltaT", "c")


def load_zaragoza(path):
    """(nlos_data [T,H,W], camera_position [3], camera_grid_size [2], camera_grid_positions [3,H*W],
    camera_grid_points [2], volume_position [3], volume_size, deltaT, c) as numpy / floats."""
    import scipy.io
    try:
        m = scipy.io.loadmat(path)
    except NotImplementedError as e:   # MATLAB v7.3 = HDF5
        raise RuntimeError(f"nlosgr: {path} is a MATLAB v7.3 (HDF5) file; reading it needs h5py") from e
    missing = [k for k in ZARAGOZA_KEYS if k not in m]
    if missing:
        raise KeyError(f"nlosgr: {path} lacks Zaragoza fields {missing}")
    data = np.asarray(m["data"], dtype=np.float32)
    while data.ndim > 3 and data.shape[0] == 1:
        data = data[0]
    if data.ndim != 3:
        raise ValueError(f"nlosgr: Zaragoza 'data' must be [T,H,W], got {data.shape}")
    flat = lambda k: np.asarray(m[k], dtype=np.float64).reshape(-1)
    grid_pos = np.asarray(m["cameraGridPositions"], dtype=np.float32)
    if grid_pos.shape[0] != 3:
        grid_pos = grid_pos.reshape(3, -1)
    return (data, flat("cameraPosition"), flat("cameraGridSize"), grid_pos, flat("cameraGridPoints"),
            flat("hiddenVolumePosition"), float(flat("hiddenVolumeSize")[0]), float(flat("deltaT")[0]),
            float(flat("c")[0]))


def save_zaragoza(path, nlos_data, camera_grid_positions, volume_position, volume_size, deltaT, c,
                  camera_position=(0.0, 0.0, 0.0), camera_grid_size=None, camera_grid_points=None):
    """Write a capture (or a rendered volume) in the same format load_zaragoza reads."""
    import scipy.io
    T, H, W = nlos_data.shape
    scipy.io.savemat(path, {
        "data": np.asarray(nlos_data, dtype=np.float32),
        "cameraPosition": np.asarray(camera_position, dtype=np.float64).reshape(1, 3),
        "cameraGridSize": np.asarray(camera_grid_size if camera_grid_size is not None else (1.0, 1.0)).reshape(1, 2),
        "cameraGridPositions": np.asarray(camera_grid_positions, dtype=np.float32).reshape(3, H * W),
        "cameraGridPoints": np.asarray(camera_grid_points if camera_grid_points is not None else (H, W)).reshape(1, 2),
        "hiddenVolumePosition": np.asarray(volume_position, dtype=np.float64).reshape(1, 3),
        "hiddenVolumeSize": np.asarray([[volume_size]], dtype=np.float64),
        "deltaT": np.asarray([[deltaT]], dtype=np.float64),
        "c": np.asarray([[c]], dtype=np.float64),
    })


@torch.no_grad()
def data_shuffle(nlos_data, camera_grid_positions, device):
    """main.py:38-57: one random permutation (torch.randperm, global generator) of the wall points,
    applied to the histograms and their positions.  Returns (nlos_data [L,M,N], camera_grid_positions
    [3, MN], index [MN] = original flat wall index of each shuffled column)."""
    L, M, N = nlos_data.shape
    nlos_data = nlos_data.reshape(L, -1)
    if not torch.is_tensor(camera_grid_positions):
        camera_grid_positions = torch.from_numpy(np.asarray(camera_grid_positions))
    camera_grid_positions = camera_grid_positions.float().to(device)
    index = torch.linspace(0, M * N - 1, M * N, dtype=torch.float, device=device).reshape(1, -1)
    full = torch.cat((nlos_data, camera_grid_positions, index), axis=0)
    full = full[:, torch.randperm(full.size(1))]
    return full[0:L, :].view(L, M, N), full[L:-1, :], full[-1, :]


def make_data_kwargs(path, device, shuffle=True):
    """main.py:90-133 over load_zaragoza: (data_kwargs, nlos_data, camera_grid_positions, index)."""
    (nlos_data, _cam_pos, grid_size, grid_pos, _grid_pts, vol_pos, vol_size, deltaT, c) = load_zaragoza(path)
    pmin = np.concatenate((vol_pos - vol_size / 2, np.array([0, -np.pi])), axis=0)
    pmax = np.concatenate((vol_pos + vol_size / 2, np.array([np.pi, 0])), axis=0)
    box = volume_box_point(tuple(float(v) for v in vol_pos), vol_size, device)
    nlos_data = torch.tensor(nlos_data, dtype=torch.float, device=device)
    L, M, N = nlos_data.shape
    if shuffle:
        nlos_data, grid_pos_t, index = data_shuffle(nlos_data, grid_pos, device)
    else:
        grid_pos_t = torch.from_numpy(grid_pos).float().to(device)
        index = torch.arange(M * N, dtype=torch.float, device=device)
    data_kwargs = {
        "nlos_data": nlos_data, "index": index, "camera_grid_positions": grid_pos_t,
        "camera_grid_size": torch.tensor(grid_size, dtype=torch.float, device=device),
        "volume_position": torch.tensor(vol_pos, dtype=torch.float, device=device), "volume_size": vol_size,
        "volume_box_point": box, "deltaT": deltaT, "c": c,
        "pmin": torch.tensor(pmin, dtype=torch.float, device=device),
        "pmax": torch.tensor(pmax, dtype=torch.float, device=device),
    }
    return data_kwargs, nlos_data, grid_pos_t, index


def volume_geometry(data_kwargs, ns, start, end, preset="cuda", mode="noocl"):
    """Batched sampling tables for every wall point of data_kwargs, in the (shuffled) column order of
    nlos_data.reshape(L, M*N): wall point v = m*N + n is column v (nlos_helpers.py:302-306)."""
    walls = data_kwargs["camera_grid_positions"].t().contiguous().float()
    vp = data_kwargs["volume_position"]
    return build_geometry(walls, data_kwargs["volume_box_point"].float(), ns, start, end, data_kwargs["c"],
                          data_kwargs["deltaT"], float(vp[1]), preset, mode)


def volume_target(data_kwargs, start, num_r):
    """[M*N, num_r] measured histograms nlos_data[I1:I1+num_r, m, n] for every wall point, I1 =
    floor(start) (nlos_helpers.py:153, :323), rows in the same order as volume_geometry."""
    d = data_kwargs["nlos_data"]
    L = d.shape[0]
    I1 = int(np.floor(start))
    if I1 < 0 or I1 + num_r > L:
        raise ValueError(f"nlosgr: bins [{I1}, {I1 + num_r}) outside the capture's {L} bins")
    return d[I1:I1 + num_r].reshape(num_r, -1).t().contiguous()
