"""Benchmark: transient volumes/sec (fwd+bwd), 100k Gaussians -> 128x128x1024 ToF bins (BASELINE.json).

One step = render the whole 128x128-wall-point x 1024-bin transient volume (32x32 angular
samples per wall point, "cuda" preset, no occlusion), MSE against gt_times x a target volume,
backward to the gradients of all six raw Gaussian parameter tensors, Adam update of the six
parameter groups (nlosgr.train.TrainStep: the reference's learn_one_iter, main.py:198-214, over
the whole volume).  Inputs are resident in HBM before the timed region.  With N ranks (one process per GPU, RCCL): every rank renders one full volume of
its own capture (same scene, distinct target), gradients are summed with one all-reduce per
step -> weak scaling, value = N volumes per step / max-over-ranks step time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3] [--cutoff 3.0]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nlos-gaussian-renderer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CONFIGS = {
    # name: (Ng, H, W, T, Ns, fwd_only)
    "C1": (1_000, 32, 32, 128, 32, False),
    "C2": (50_000, 64, 64, 512, 32, True),
    "C3": (100_000, 128, 128, 1024, 32, False),
    "C5": (500_000, 256, 256, 2048, 32, False),
    "S1": (20_000, 32, 32, 512, 32, False),      # quick iteration size (not a BASELINE config)
}
PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_FP32_TFLOPS = 157.3       # FP32 vector peak (the path has no MFMA shape)
FLOP_PER_EVAL = {"fwd": 36, "bwd": 100}   # SURVEY §8d convention (FMA = 2, exp = 1)


def param_bytes(deg):
    return 4 * (3 + 3 + 4 + 1 + (deg + 1) ** 2)        # 108 B at SH degree 3


def cpu_baseline(cfg_name, seed=0, preset="cuda", mode="noocl"):
    """Time the CPU oracle (dense restatement of the reference path, same preset and mode as the GPU run) on a
    bounded sample of the same workload: 1 wall point x G_SAMPLE of the Ng Gaussians x the full
    Ns^2 x T sample grid, fwd+bwd, in chunks of 32 Gaussians (bounded memory); extrapolated
    linearly (the dense cost is linear in Gaussians and in wall points)."""
    from nlosgr.model import GaussianParams
    from nlosgr.volume import Scene
    from oracle import torch_ref as R
    ng, H, W, T, ns, _ = CONFIGS[cfg_name]
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    scene = Scene(H=H, W=W, T=T, ns=ns)
    g_sample = max(1, min(ng, int(os.environ.get("NLOSGR_CPU_SAMPLE_G", "160"))))
    m = GaussianParams.synthetic(ng, 3, preset=preset, device="cpu", seed=seed)
    walls = scene.walls("cpu")
    p = walls[(H // 2) * W + W // 2]
    tab = R.sample_tables(p, scene.box("cpu"), ns, scene.start, scene.end, scene.c, scene.deltaT)
    t0 = time.perf_counter()
    for g0 in range(0, g_sample, 32):
        sl = slice(g0, min(g_sample, g0 + 32))
        P = R.Params(*(t.detach()[sl].clone() for t in (m._mu, m._scaling, m._rotation, m._opacity,
                                                        m._features_dc, m._features_rest)), 3)
        _, h = R.render_wallpoint(P, p, tab, 0.5, scene.c, scene.deltaT, preset=preset, mode=mode)
        (h * h).sum().backward()
    t = time.perf_counter() - t0
    per_volume = t * (ng / g_sample) * (H * W)
    return {"value": 1.0 / per_volume, "unit": "volumes/s", "cores": threads, "kind": "port",
            "sample": f"oracle/torch_ref dense ({preset} preset, {mode}) fwd+bwd of 1 wall point x {g_sample} of {ng} "
                      f"Gaussians x {ns}x{ns}x{T} samples = {t:.2f} s on {threads} threads; "
                      f"extrapolated x{ng / g_sample:g} Gaussians x{H * W} wall points"}


def pmc_traffic(cfg_name, kernels):
    """HBM bytes per launch of `kernels` (name substrings) from the newest committed
    profiles/r*_<cfg>_traffic.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes of this bench,
    scripts/prof_c3.sh + scripts/summarize_prof.py), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{cfg_name.lower()}_traffic.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        rec = json.load(f)["kernels"]
    total = 0.0
    for sub in kernels:
        hits = [v["hbm_bytes_per_launch"] for k, v in rec.items() if sub in k]
        if not hits:
            return None, None
        total += max(hits)
    return total, os.path.relpath(files[-1], ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--cutoff", type=float, default=3.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-json", default="")
    ap.add_argument("--preset", default="cuda", choices=("cuda", "torch"),
                    help="convention preset: cuda = the reference's CUDA path, torch = its torch path (SURVEY A.3)")
    ap.add_argument("--mode", default="noocl", choices=("noocl", "netf"),
                    help="rendering_type: noocl (configs/default.py:15 default) or netf self-transmittance")
    ap.add_argument("--band", type=int, default=0,
                    help="render only wall band 0 of BAND equal bands (one rank's share of a BAND-GPU sharded "
                         "volume, nlosgr.distributed.wall_band); value = projected volumes/s of the sharded job")
    ap.add_argument("--shard", action="store_true",
                    help="with N ranks, rank r renders wall band r of N (SURVEY §8e: one volume per step over "
                         "the whole job, packed gradient all-reduce timed) -> strong scaling")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # NLOSGR_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (rank -> GPU local % count); the
    # production path is RCCL ("nccl"), one GPU per rank
    ndev = max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local % ndev)
        dist.init_process_group(os.environ.get("NLOSGR_DIST_BACKEND", "nccl"))
    dev = torch.device("cuda", local % ndev)

    from nlosgr import GaussianParams
    from nlosgr.model import features_flat
    from nlosgr.render import render_forward
    from nlosgr.train import TrainStep
    from nlosgr.volume import Scene, make_config

    ng, H, W, T, ns, fwd_only = CONFIGS[a.config]
    scene = Scene(H=H, W=W, T=T, ns=ns)
    model = GaussianParams.synthetic(ng, 3, preset=a.preset, device=dev, seed=0)
    nwall = H * W
    if a.shard and world > 1 and a.band > 1:
        raise SystemExit("--band is a single-GPU projection; with N ranks use --shard")
    band_n, band_r = (world, rank) if (a.shard and world > 1) else (a.band, 0)
    if band_n > 1:   # one rank's contiguous band of the wall (SURVEY §8e sharding)
        from nlosgr.distributed import wall_band
        b0, b1 = wall_band(H * W, band_r, band_n)
        geo = scene.geometry(dev, a.preset, a.mode, walls=scene.walls(dev)[b0:b1].contiguous())
        nwall = b1 - b0
    else:
        geo = scene.geometry(dev, a.preset, a.mode)
    cfg = make_config(model, scene, a.preset, a.mode, cutoff=a.cutoff)
    g = torch.Generator().manual_seed(1 + rank)
    target = (torch.rand(nwall, T, generator=g) * 1e-3).to(dev)   # measured volume, x gt_times=100 in the loss
    ev_fwd = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev_bwd = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fwd_ms, bwd_ms = [], []
    # one training iteration of the reference (main.py:198-214) over the whole volume, fused on the
    # device: forward (records the ray cache) -> MSE vs gt_times * target + dL/dhist -> backward
    # (walks the ray cache) -> [packed gradient all-reduce] -> Adam over the six parameter groups
    train = TrainStep(model, geo, cfg, target, gt_times=100.0, nwall_total=H * W if band_n > 1 else H * W * world,
                      events={"fwd": ev_fwd, "bwd": ev_bwd})
    stream = torch.cuda.current_stream(dev)

    def step(timed):
        if fwd_only:
            params = [model._mu.detach(), model._scaling.detach(), model._rotation.detach(),
                      model._opacity.detach(), features_flat(model).detach().contiguous()]
            ev_fwd[0].record(stream)
            hist, _ = render_forward(*params, geo, cfg, True, False)
            ev_fwd[1].record(stream)
            return hist
        return train()

    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
        torch.cuda.synchronize(dev)
        fwd_ms.append(ev_fwd[0].elapsed_time(ev_fwd[1]))
        if not fwd_only:
            bwd_ms.append(ev_bwd[0].elapsed_time(ev_bwd[1]))
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms_per_step = elapsed * 1000.0 / a.steps
    # weak (replicas): every rank finishes one volume per step; sharded: the job finishes one
    volumes_per_s = (1 if a.shard and world > 1 else world) * a.steps / elapsed

    # roofline of the dominant phase (algorithmic HBM bytes / measured launch time)
    pb = param_bytes(3)
    V = 4 * nwall * T
    fwd_avg = sum(fwd_ms) / len(fwd_ms)
    bwd_avg = sum(bwd_ms) / len(bwd_ms) if bwd_ms else 0.0
    if bwd_avg >= fwd_avg:
        dom, dom_ms, dom_bytes = "bwd", bwd_avg, 2 * ng * pb + V
        kern = ("preprocess_kernel", "bwd_kernel", "sh_kernel", "finish_kernel")
    else:
        dom, dom_ms, dom_bytes = "fwd", fwd_avg, ng * pb + V
        kern = ("preprocess_kernel", "fwd_kernel")
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(a.config, kern)
    # secondary roofline: in-support evaluations (counting pass, untimed) x SURVEY FLOP convention
    from nlosgr.render import count_support
    params = [model._mu.detach(), model._scaling.detach(), model._rotation.detach(), model._opacity.detach(),
              features_flat(model).detach().contiguous()]
    pairs, rays, evals = count_support(*params, geo, cfg)
    flops = evals * FLOP_PER_EVAL[dom]
    valu = {"bound": "valu", "evaluations": evals, "pairs": pairs, "rays": rays,
            "flop_per_eval": FLOP_PER_EVAL[dom], "achieved": flops / (dom_ms * 1e-3) / 1e12,
            "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s"}
    valu["frac"] = valu["achieved"] / PEAK_FP32_TFLOPS
    out = {
        "metric": "transient volumes/sec (fwd+bwd), 100k Gaussians → 128×128×1024 ToF bins"
        if a.config == "C3" and (a.preset, a.mode) == ("cuda", "noocl") else f"transient volumes/sec ({'fwd' if fwd_only else 'fwd+bwd'}) {a.config}",
        "value": volumes_per_s, "unit": "volumes/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "strong" if a.shard and world > 1 else "weak", "vs_baseline": None,
        "dtype": "f32", "data": "synthetic (SURVEY §8d geometry, seeded random Gaussians and target)",
        "config": {"workload": f"{a.config}: {ng} Gaussians -> {H}x{W} wall x {T} bins, {ns}x{ns} angular "
                               f"samples, {a.preset} preset, {'no occlusion' if a.mode == 'noocl' else a.mode}, "
                               f"{'dense (every sample)' if a.cutoff <= 0 else f'support cutoff {a.cutoff} sigma'}, "
                               f"{'fwd' if fwd_only else 'fwd+MSE+bwd (6 param grads)+Adam'}",
                   "gaussians": ng, "wall": [H, W], "bins": T, "angular": ns, "cutoff": a.cutoff,
                   "preset": a.preset, "mode": a.mode,
                   "parallelism": (f"wall shard: {world} bands (rank r renders band r), packed grad "
                                   f"all-reduce" if a.shard and world > 1 else
                                   f"one rank's band of a {a.band}-way wall shard (projected job rate; the "
                                   f"packed gradient all-reduce is not timed)" if a.band > 1 else
                                   f"wall-replica x{world}, grad all-reduce" if world > 1 else "single GPU")},
        "phase_ms": {"fwd": fwd_avg, "bwd": bwd_avg},
        "roofline": {"bound": "hbm", "kernel": f"nlosgr {dom} ({' + '.join(kern)})", "achieved": achieved,
                     "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_ms": dom_ms},
        "roofline_valu": valu,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(a.config, preset=a.preset, mode=a.mode)
        except Exception as e:  # report, never fake
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
