"""MCMC relocation rule (nlosgr.densify.compute_relocation, 3DGS-MCMC eqs. 9-10 as its
compute_relocation kernel evaluates them): identity at N = 1, the N copies' composed opacity
equals the original, and the double sum of the published kernel equals the single-sum form used
here.  Parity unpinned (the reference's densification cannot run)."""
import math

import torch


def _double_sum(o, s, N):
    o_new = 1.0 - (1.0 - o) ** (1.0 / N)
    den = 0.0
    for i in range(1, N + 1):
        for k in range(i):
            den += math.comb(i - 1, k) * ((-1) ** k / math.sqrt(k + 1)) * o_new ** (k + 1)
    return o_new, s * o / den


def test_identity_at_one_copy():
    from nlosgr.densify import compute_relocation
    o = torch.tensor([0.3, 0.9, 0.01])
    s = torch.rand(3, 3) + 0.1
    o2, s2 = compute_relocation(o, s, torch.ones(3, dtype=torch.long))
    torch.testing.assert_close(o2, o)
    torch.testing.assert_close(s2, s)


def test_opacity_composition_and_published_double_sum():
    from nlosgr.densify import compute_relocation
    o = torch.tensor([0.2, 0.5, 0.95, 0.7], dtype=torch.float64)
    s = torch.tensor([[0.1, 0.2, 0.3]] * 4, dtype=torch.float64)
    N = torch.tensor([2, 3, 5, 9])
    o2, s2 = compute_relocation(o, s, N)
    torch.testing.assert_close(1 - (1 - o2) ** N.double(), o)
    for i in range(4):
        eo, es = _double_sum(float(o[i]), s[i].numpy(), int(N[i]))
        assert abs(float(o2[i]) - eo) < 1e-12
        assert abs(float(s2[i, 0]) - es[0]) < 1e-9 * abs(es[0])


def test_relocate_moves_dead_onto_live_cpu():
    from nlosgr import GaussianParams
    from nlosgr.densify import prune_dead_mask, relocate_gs
    torch.manual_seed(0)
    m = GaussianParams.synthetic(64, 3, preset="cuda", device="cpu", seed=2)
    m._opacity.data[:8] = -12.0                       # dead: sigmoid < 0.005
    dead = prune_dead_mask(m)
    assert int(dead.sum()) == 8
    relocate_gs(m, dead)
    assert int(prune_dead_mask(m).sum()) == 0
    # every relocated Gaussian sits on a live Gaussian's position
    live_mu = m._mu.data[8:]
    d = (m._mu.data[:8, None, :] - live_mu[None]).abs().amax(-1).amin(1)
    assert (d == 0).all()
