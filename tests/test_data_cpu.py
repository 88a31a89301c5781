"""Captured-data path and checkpoints on CPU (no GPU): Zaragoza .mat round trip, the reference's
data_shuffle semantics (main.py:38-57), whole-volume targets / geometry, and checkpoint keys
loadable with torch.load(weights_only=True).  The Zaragoza format has no fixture in the
reference (its loader module is absent): parity unpinned, round-trip tested."""
import numpy as np
import pytest
import torch


def _capture(T=40, H=3, W=4, seed=0):
    g = np.random.default_rng(seed)
    data = g.random((T, H, W)).astype(np.float32)
    xs = np.linspace(-0.5, 0.5, W)
    zs = np.linspace(-0.5, 0.5, H)
    pos = np.stack([np.repeat(xs[None, :], H, 0).reshape(-1), np.zeros(H * W), np.repeat(zs[:, None], W, 1).reshape(-1)])
    return data, pos.astype(np.float32)


def test_zaragoza_round_trip(tmp_path):
    from nlosgr.data import load_zaragoza, save_zaragoza
    data, pos = _capture()
    f = tmp_path / "cap.mat"
    save_zaragoza(str(f), data, pos, (0.0, 0.5, 0.0), 0.5, 0.01, 1.0)
    out = load_zaragoza(str(f))
    assert len(out) == 9
    np.testing.assert_array_equal(out[0], data)
    np.testing.assert_array_equal(out[3], pos)
    np.testing.assert_allclose(out[5], [0.0, 0.5, 0.0])
    assert out[6] == 0.5 and out[7] == 0.01 and out[8] == 1.0


def test_zaragoza_missing_field(tmp_path):
    import scipy.io
    from nlosgr.data import load_zaragoza
    f = tmp_path / "bad.mat"
    scipy.io.savemat(str(f), {"data": np.zeros((2, 2, 2))})
    with pytest.raises(KeyError):
        load_zaragoza(str(f))


def test_data_shuffle_is_a_consistent_permutation():
    from nlosgr.data import data_shuffle
    data, pos = _capture()
    L, M, N = data.shape
    torch.manual_seed(3)
    d2, p2, idx = data_shuffle(torch.from_numpy(data), pos, "cpu")
    assert d2.shape == (L, M, N) and p2.shape == (3, M * N) and idx.shape == (M * N,)
    perm = idx.long()
    assert sorted(perm.tolist()) == list(range(M * N))
    np.testing.assert_array_equal(d2.reshape(L, -1).numpy(), data.reshape(L, -1)[:, perm.numpy()])
    np.testing.assert_array_equal(p2.numpy(), pos[:, perm.numpy()])
    # same generator state -> same permutation (torch.randperm of main.py:46)
    torch.manual_seed(3)
    expect = torch.randperm(M * N)
    torch.manual_seed(3)
    _, _, idx2 = data_shuffle(torch.from_numpy(data), pos, "cpu")
    np.testing.assert_array_equal(idx2.long().numpy(), expect.numpy())


def test_volume_target_and_geometry(tmp_path):
    from nlosgr.data import make_data_kwargs, save_zaragoza, volume_geometry, volume_target
    data, pos = _capture(T=64)
    f = tmp_path / "cap.mat"
    save_zaragoza(str(f), data, pos, (0.0, 0.5, 0.0), 0.5, 1.28 / 48, 1.0)
    torch.manual_seed(0)
    dk, nd, gp, idx = make_data_kwargs(str(f), "cpu")
    start, end = 6, 6 + 48
    tgt = volume_target(dk, start, end - start)
    M, N = data.shape[1:]
    assert tgt.shape == (M * N, 48)
    v = 5
    m, n = divmod(v, N)
    np.testing.assert_array_equal(tgt[v].numpy(), nd[start:start + 48, m, n].numpy())   # nlos_helpers.py:302-324
    geo = volume_geometry(dk, 4, start, end, "cuda")
    assert geo.nwall == M * N and geo.nr == 48
    np.testing.assert_allclose(geo.wall.numpy(), gp.t().numpy())
    with pytest.raises(ValueError):
        volume_target(dk, 40, 48)


def test_checkpoint_round_trip_weights_only(tmp_path):
    from nlosgr import GaussianParams
    from nlosgr.checkpoint import PARAM_KEYS, load_checkpoint, save_checkpoint
    m = GaussianParams.synthetic(50, 3, preset="cuda", device="cpu", seed=1)
    m.active_sh_degree = 2
    f = tmp_path / "ck.pt"
    save_checkpoint(str(f), m)
    raw = torch.load(str(f), weights_only=True)
    assert set(PARAM_KEYS) <= set(raw) and raw["max_sh_degree"] == 3 and raw["active_sh_degree"] == 2
    m2 = load_checkpoint(str(f))
    for k in PARAM_KEYS:
        assert torch.equal(getattr(m, "_" + k).detach(), getattr(m2, "_" + k).detach())
    assert m2.active_sh_degree == 2 and m2.max_sh_degree == 3
