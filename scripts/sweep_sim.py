"""Design simulation (CPU, numpy): lane efficiency of window-sweep forward drains on real C3 segments.

Generates the (kl, kh) ray segments of one C3 wall point at 5.7 sigma for chunks of 64 Gaussians
(the kernel's per-wave unit), in index order or in Morton order, and replays sweep policies:
lanes of one wave share a window of S bins; a free lane can take a pending segment only at a window
boundary W and only if its start lies in [W, W + G); the window advances by S while any lane is
busy, otherwise jumps to the earliest pending start.  Efficiency = in-segment bins / (64 x slots).
    python scripts/sweep_sim.py [--wall 0.5,0.5] [--chunks 8] [--morton]
"""
import argparse
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlos-gaussian-renderer_amd"))
sys.path.insert(0, ROOT)


def segments(ng=100_000, wall_uv=(0.5, 0.5), chunk=64, nchunks=8, morton=False, mc=5.7, seed=0):
    from nlosgr.model import GaussianParams
    from nlosgr.volume import Scene
    from oracle.torch_ref import quat_to_rotmat_cuda
    scene = Scene(H=128, W=128, T=1024, ns=32)
    geo = scene.geometry("cpu", "cuda")
    H = W = 128
    p = int(wall_uv[0] * (H - 1)) * W + int(wall_uv[1] * (W - 1))
    m = GaussianParams.synthetic(ng, 3, preset="cuda", device="cpu", seed=seed)
    mu = m._mu.detach().double().numpy()
    s = np.exp(m._scaling.detach().double().numpy())
    R = quat_to_rotmat_cuda(m._rotation.detach()).double().numpy()     # [ng,3,3]
    order = np.arange(ng)
    if morton:
        q = ((mu - mu.min(0)) / (mu.max(0) - mu.min(0) + 1e-9) * 1023).astype(np.int64)
        def spread(x):
            x &= 0x3FF
            x = (x | (x << 16)) & 0x030000FF
            x = (x | (x << 8)) & 0x0300F00F
            x = (x | (x << 4)) & 0x030C30C3
            x = (x | (x << 2)) & 0x09249249
            return x
        order = np.argsort(spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2), kind="stable")
    wall = geo.wall[p].double().numpy()
    st, ct = geo.sin_theta[p].double().numpy(), geo.cos_theta[p].double().numpy()
    sp, cp = geo.sin_phi[p].double().numpy(), geo.cos_phi[p].double().numpy()
    d = np.stack([(st[:, None] * cp[None, :]).ravel(), (st[:, None] * sp[None, :]).ravel(),
                  np.repeat(ct, len(cp))], 1)                             # [1024,3]
    r = geo.r.double().numpy()
    r0, dr, nr = r[0], r[1] - r[0], len(r)
    out = []
    rng = np.random.default_rng(1)
    picks = rng.choice(ng // chunk, nchunks, replace=False)
    for c in picks:
        idx = order[c * chunk:(c + 1) * chunk]
        A = R[idx].transpose(0, 2, 1) / (s[idx][:, :, None] + 1e-8)        # u = R^T (x - mu) / s
        u0 = np.einsum("gij,gj->gi", A, wall[None, :] - mu[idx])
        v = np.einsum("gij,rj->gri", A, d)                                  # [g,1024,3]
        a = (v * v).sum(-1)
        ts = -(u0[:, None, :] * v).sum(-1) / a
        zs = u0[:, None, :] + ts[..., None] * v
        m2 = (zs * zs).sum(-1)
        ok = m2 <= mc * mc
        ks = (ts - r0) / dr
        hk = np.sqrt(np.maximum(mc * mc - m2, 0) / a) / dr
        kl = np.clip(np.ceil(ks - hk), 0, nr).astype(int)
        kh = np.clip(np.floor(ks + hk), -1, nr - 1).astype(int)
        ok &= kl <= kh
        ga = -0.5 / math.log(2) * a * dr * dr
        seg = np.stack([kl[ok], kh[ok], ga[ok], ks[ok]], 1)
        out.append(seg)
    return out


def simulate(seg, S=32, G=8, late=False):
    """One wave, 64 lanes: returns (efficiency, slots, useful).  late: a free lane with nothing
    eligible takes the body [W, kh] of a pending segment that started before W (its head [kl, W)
    stays pending as a shorter segment)."""
    order = np.argsort(seg[:, 0], kind="stable")
    kl = seg[order, 0].astype(int)
    kh = seg[order, 1].astype(int)
    taken = np.zeros(len(kl), bool)
    lane_end = np.full(64, -1)           # last bin of the lane's segment
    Wb = kl.min() if len(kl) else 0
    slots = 0
    useful = int((kh - kl + 1).sum())
    while not taken.all() or (lane_end >= Wb).any():
        free = np.where(lane_end < Wb)[0]
        if len(free) and not taken.all():
            elig = np.where(~taken & (kl >= Wb) & (kl < Wb + G))[0][:len(free)]
            for l, e in zip(free, elig):
                taken[e] = True
                lane_end[l] = kh[e]
            if late and len(free) > len(elig):
                lt = np.where(~taken & (kl < Wb) & (kh >= Wb + S))[0]
                lt = lt[np.argsort(-kl[lt], kind="stable")][:len(free) - len(elig)]
                for l, e in zip(free[len(elig):], lt):
                    lane_end[l] = kh[e]
                    kh[e] = Wb - 1             # the head stays pending
        if not (lane_end >= Wb).any():
            if taken.all():
                break
            Wb = kl[~taken].min()        # all lanes idle: jump to the earliest pending start
            lane_end[:] = -1
            continue
        slots += S
        Wb += S
    return useful / max(1, 64 * slots), slots, useful


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--wall", default="0.5,0.5")
    ap.add_argument("--chunks", type=int, default=6)
    ap.add_argument("--chunk", type=int, default=64)
    ap.add_argument("--morton", action="store_true")
    a = ap.parse_args()
    wu = tuple(float(x) for x in a.wall.split(","))
    segs = segments(wall_uv=wu, chunk=a.chunk, nchunks=a.chunks, morton=a.morton)
    n = [len(x) for x in segs]
    L = np.concatenate([x[:, 1] - x[:, 0] + 1 for x in segs])
    span = [int(x[:, 0].max() - x[:, 0].min()) if len(x) else 0 for x in segs]
    print(f"segments per chunk {n}, mean len {L.mean():.1f}, start span per chunk {span}")
    for S, G, late in ((16, 16, False), (16, 16, True), (8, 8, False), (8, 8, True), (32, 32, True)):
        effs = [simulate(x, S, G, late)[0] for x in segs if len(x)]
        print(f"S={S:3d} G={G:3d} late={late}: efficiency {np.mean(effs):.3f} (per chunk {', '.join(f'{e:.2f}' for e in effs)})")


def simulate_groups(seg, S=16, ngroups=4, late=True):
    """ngroups sweepers of 64/ngroups lanes in lockstep (each its own window base), one shared
    pending pool; late-taking as in simulate()."""
    order = np.argsort(seg[:, 0], kind="stable")
    kl = seg[order, 0].astype(int)
    kh = seg[order, 1].astype(int).copy()
    useful = int((kh - kl + 1).sum())
    lanes = 64 // ngroups
    taken = np.zeros(len(kl), bool)
    ends = np.full((ngroups, lanes), -1)
    Wg = np.zeros(ngroups, dtype=np.int64)
    steps = 0
    while True:
        if taken.all() and all((ends[g] < Wg[g]).all() for g in range(ngroups)):
            break
        for g in range(ngroups):
            W = Wg[g]
            if (ends[g] < W).all():                  # idle group: jump to the earliest pending start
                if taken.all():
                    continue
                W = Wg[g] = kl[~taken].min()
                ends[g][:] = -1
            free = np.where(ends[g] < W)[0]
            if len(free) and not taken.all():
                elig = np.where(~taken & (kl >= W) & (kl < W + S))[0][:len(free)]
                for l, e in zip(free, elig):
                    taken[e] = True
                    ends[g][l] = kh[e]
                if late and len(free) > len(elig):
                    lt = np.where(~taken & (kl < W) & (kh >= W + S))[0]
                    lt = lt[np.argsort(-kl[lt], kind="stable")][:len(free) - len(elig)]
                    for l, e in zip(free[len(elig):], lt):
                        ends[g][l] = kh[e]
                        kh[e] = W - 1
        steps += 1
        Wg += S
    return useful / max(1, 64 * S * steps)


def main_groups():
    segs = segments(chunk=int(os.environ.get("SIM_CHUNK", "64")), nchunks=3)
    for S, ng in ((16, 1), (16, 2), (16, 4), (8, 4), (16, 8)):
        effs = [simulate_groups(x, S, ng) for x in segs]
        print(f"S={S} groups={ng}: efficiency {np.mean(effs):.3f}")
