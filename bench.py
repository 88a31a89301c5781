"""Benchmark: transient volumes/sec (fwd+bwd), 100k Gaussians -> 128x128x1024 ToF bins (BASELINE.json).

One step = one training iteration of the reference (main.py:198-214 learn_one_iter) over the whole
128x128-wall-point x 1024-bin transient volume (32x32 angular samples per wall point, "cuda"
preset, no occlusion): render forward (records the ray cache) -> MSE against gt_times x a target
volume + dL/dhist -> backward to all six raw Gaussian parameter tensors -> Adam on the six groups
(nlosgr.train.TrainStep).  Inputs are resident in HBM before the timed region.

Frozen workload: every step (warm-up and timed) first restores the parameters, the Adam moments and
the iteration counter from one device snapshot (a ~34 MB device copy inside the timed region), so
each timed step renders exactly the same Gaussians; the in-support evaluation count reported is that
of the snapshot, i.e. of every step.

Default cutoff 5.7 sigma = the parity-grade support (pdf < 1e-7 of the peak dropped;
rel-L2 vs the 6-sigma volume 1e-7).  `--lines 3.0` adds the same step at 3 sigma (the reference
CUDA path's sigma_threshold; rel-L2 vs dense ~3e-2) under `lines` for comparison; never `value`.

With N ranks (one process per GPU, RCCL): the relay wall is split into N shards of whole wall rows,
row-interleaved (rank r renders rows r, r+N, ...: balanced work, nlosgr.distributed.wall_rows), and
the packed gradients are summed with one bucketed all-reduce per step ->
strong scaling, value = 1 volume per step / max-over-ranks step time.  --replicas instead gives
every rank a full volume of its own capture (weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3] [--cutoff 5.7] [--lines 3.0] [--band 8] [--replicas]

Launch: under a launcher (torch.distributed.run: WORLD_SIZE set) every process is one rank and
WORLD_SIZE must equal --gpus.  Without one, `--gpus N` > 1 starts N fresh child interpreters of this
script itself (rank r -> GPU r, RCCL over xGMI, rendezvous on 127.0.0.1) BEFORE anything touches the
GPU, waits for them and exits with the worst exit code; rank 0's line is the job's line.
NLOSGR_BENCH_STUB=1 replaces the render step by a small CPU step (gloo) so the launcher, the barriers
and the max-over-ranks timing can be rehearsed without a GPU (tests/test_bench_launch_cpu.py).
"""
import argparse
from dataclasses import replace
import json
import os
import socket
import statistics
import subprocess
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
PROGRESS = os.environ.get("NLOSGR_BENCH_PROGRESS") == "1"   # per-step lines on stderr (long profiled runs)
PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def param_bytes(deg):
    return 4 * (3 + 3 + 4 + 1 + (deg + 1) ** 2)        # 108 B at SH degree 3


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cfg_name, cutoff, seed=0, preset="cuda", mode="noocl"):
    """The CPU oracle (oracle/torch_ref: the reference's dense torch path restated, same preset, mode
    and support cutoff as the GPU run, so its outputs are the GPU's) on a bounded sample of the same
    workload: WALLS wall points x G_SAMPLE of the Ng Gaussians x the full Ns^2 x T sample grid,
    fwd+bwd.  One warm-up, then the median of 3 timed runs, on every host thread this process may
    use (OMP_NUM_THREADS on the GPU box = its CPU share); extrapolated linearly in Gaussians and
    wall points (the dense cost is linear in both)."""
    from nlosgr.model import GaussianParams
    from nlosgr.volume import Scene
    from oracle import torch_ref as R
    ng, H, W, T, ns, _ = CONFIGS[cfg_name]
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    scene = Scene(H=H, W=W, T=T, ns=ns)
    g_sample = max(1, min(ng, int(os.environ.get("NLOSGR_CPU_SAMPLE_G", "64"))))
    m = GaussianParams.synthetic(ng, 3, preset=preset, device="cpu", seed=seed)
    walls = scene.walls("cpu")
    pick = [(H // 4) * W + W // 4, (3 * H // 4) * W + 3 * W // 4]
    tabs = [(walls[i], R.sample_tables(walls[i], scene.box("cpu"), ns, scene.start, scene.end, scene.c,
                                       scene.deltaT)) for i in pick]
    # spread the sample over the index range (synthetic Gaussians are i.i.d., so any subset is typical)
    idx = torch.linspace(0, ng - 1, g_sample).long()
    mc = cutoff if cutoff > 0 else None

    def run():
        t0 = time.perf_counter()
        for g0 in range(0, g_sample, 32):
            sl = idx[g0:g0 + 32]
            P = R.Params(*(t.detach()[sl].clone() for t in (m._mu, m._scaling, m._rotation, m._opacity,
                                                            m._features_dc, m._features_rest)), 3)
            for p, tab in tabs:
                _, h = R.render_wallpoint(P, p, tab, 0.5, scene.c, scene.deltaT, preset=preset, mode=mode, mc=mc)
                (h * h).sum().backward()
        return time.perf_counter() - t0

    run()                                   # warm-up
    times = [run() for _ in range(3)]
    t = statistics.median(times)
    per_volume = t * (ng / g_sample) * (H * W / len(pick))
    return {"value": 1.0 / per_volume, "unit": "volumes/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"oracle/torch_ref dense ({preset} preset, {mode}, cutoff mask {cutoff} sigma) fwd+bwd of "
                      f"{len(pick)} wall points x {g_sample} of {ng} Gaussians x {ns}x{ns}x{T} samples: median "
                      f"of 3 after 1 warm-up = {t:.2f} s (runs {', '.join(f'{x:.2f}' for x in times)}) on "
                      f"{threads} threads; extrapolated x{ng / g_sample:g} Gaussians x{H * W / len(pick):g} wall "
                      f"points"}


def committed_profile(cfg_name, kind, cutoff, preset="cuda", mode="noocl", selection="support"):
    """The newest committed profiles/r*_<cfg>_<kind>.json (written by scripts/summarize_prof.py from
    rocprofv3 passes of this bench command) recorded for the same workload (cutoff, preset, mode,
    selection; records without those keys are the default cuda / noocl / support workload), or
    (None, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{cfg_name.lower()}_{kind}.json")))
    for fn in reversed(files):
        with open(fn) as f:
            rec = json.load(f)
        if (rec.get("cutoff") == cutoff and rec.get("preset", "cuda") == preset and rec.get("mode", "noocl") == mode
                and rec.get("selection", "support") == selection):
            return rec, os.path.relpath(fn, ROOT)
    return None, None


# the kernels each timed phase launches (families: the kernel's name without template arguments);
# preprocess_kernel runs once in each phase
PHASE_KERNELS = {
    "fwd": ("preprocess_kernel", "fx_bound_kernel", "fx_unit_kernel", "fwd_kernel", "fwd_dense_kernel",
            "fx_reduce_kernel", "hist_reduce_kernel"),
    "bwd": ("preprocess_kernel", "bwd_kernel", "sh_kernel", "finish_kernel"),
    "tiles_fwd": ("preprocess_kernel", "cull_prep_kernel", "tile_cone_kernel", "tile_bin_kernel", "tile_kernel",
                  "tiles_reduce_kernel"),
    "tiles_bwd": ("preprocess_kernel", "cull_prep_kernel", "tile_cone_kernel", "tile_bin_kernel", "tile_kernel",
                  "tiles_finish_kernel"),
}
# kernels both phases launch (the same names in the profile): half their launches per step count per phase
SHARED_KERNELS = ("preprocess_kernel", "cull_prep_kernel", "tile_cone_kernel", "tile_bin_kernel")


def kernel_family(name):
    """'void fwd_kernel<1, 0, ...>' -> 'fwd_kernel' (the traffic profiles' short names)."""
    n = name[5:] if name.startswith("void ") else name
    return n.split("<", 1)[0].strip()


def rec_has_count(kernels):
    return any(kernel_family(k) == "count_kernel" for k in kernels)


def phase_traffic(kernels, phase):
    """HBM bytes per step of one timed phase from a traffic profile's per-kernel records: every kernel
    of the phase's families (the untimed support count runs as count_kernel, a family of its own, so it
    is left out by name whatever the profile's step count), each at its launches per step (a kernel of
    both phases counts half of them per phase); the ray-tile engine's tile_kernel<SEL, DENSE, OCCL, BWD>
    is split by its BWD argument.  Returns (bytes, [kernel names]) or (None, [])."""
    fams = PHASE_KERNELS[phase]
    total, used = 0.0, []
    for k, v in kernels.items():
        fam = kernel_family(k)
        if fam not in fams:
            continue
        if fam == "fwd_kernel" and v.get("launches_per_step", 1.0) < 0.5 and not rec_has_count(kernels):
            continue   # profiles older than count_kernel: the support count was a once-per-run fwd_kernel
        if fam == "tile_kernel" and k.rstrip().endswith("true>") != (phase == "tiles_bwd"):
            continue
        per = v["hbm_bytes_per_launch"]
        lps = v.get("launches_per_step", 1.0)
        total += per * (0.5 * lps if fam in SHARED_KERNELS else lps)
        used.append(k)
    return (total, used) if used else (None, [])


def pmc_traffic(cfg_name, cutoff, tiles, **wl):
    """HBM bytes per step of the forward and backward phases: FETCH_SIZE x2 + WRITE_SIZE passes
    (MI355X_MICROARCH.md §HBM) from the committed traffic profile of the same workload, or Nones."""
    rec, src = committed_profile(cfg_name, "traffic", cutoff, **wl)
    if rec is None:
        return {"fwd": None, "bwd": None}, None
    out = {}
    for ph in ("fwd", "bwd"):
        out[ph] = phase_traffic(rec["kernels"], ("tiles_" + ph) if tiles else ph)[0]
    return out, src


class Snapshot:
    """Device copy of the trainable state (six parameter tensors, Adam moments, counters)."""

    def __init__(self, train):
        self.train = train
        self.params = [t.clone() for t in train._tensors]
        self.m1 = [t.clone() for t in train.adam.exp_avg]
        self.m2 = [t.clone() for t in train.adam.exp_avg_sq]
        self.count, self.iteration = train.adam.step_count, train.iteration

    def restore(self):
        tr = self.train
        for dst, src in zip(tr._tensors, self.params):
            dst.copy_(src)
        for dst, src in zip(tr.adam.exp_avg, self.m1):
            dst.copy_(src)
        for dst, src in zip(tr.adam.exp_avg_sq, self.m2):
            dst.copy_(src)
        tr.adam.step_count, tr.iteration = self.count, self.iteration


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def timed_run(step, steps, warmup, world, dev):
    """W untimed steps, then EXACTLY K steps between barrier + synchronize on both sides; returns
    the max-over-ranks wall time, this rank's own wall time and each step's (fwd_ms, bwd_ms) from
    its HIP events (step() returns a callable read after the per-step synchronize, which the
    driver's contract keeps inside the timed region)."""
    for _ in range(warmup):
        step()
    _sync(dev)
    if world > 1:
        dist.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    phases = []
    for i in range(steps):
        phase = step()
        _sync(dev)
        phases.append(phase())
        if PROGRESS:
            print(f"[bench] step {i + 1}/{steps} fwd {phases[-1][0]:.1f} ms bwd {phases[-1][1]:.1f} ms",
                  file=sys.stderr, flush=True)
    if world > 1:
        dist.barrier()
    _sync(dev)
    own = elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    return elapsed, own, phases


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`--gpus N` without a launcher: N fresh interpreters of this script, rank r on GPU r (the
    torch.distributed.run environment: RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1,
    MASTER_PORT).  Called before anything initialises the GPU, so the parent never holds a device
    context.  If a rank fails the others are ended (they would wait at a barrier forever); the exit
    code is the worst rank's."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    codes = [None] * n
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
        if any(c not in (None, 0) for c in codes):
            for i, p in enumerate(procs):
                if codes[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if codes[i] is None:
                    try:
                        codes[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        codes[i] = p.wait()
            break
        time.sleep(0.2)
    bad = [c for c in codes if c != 0]
    if bad:
        print(f"[bench] rank exit codes {codes}", file=sys.stderr, flush=True)
        return max((abs(c) for c in bad), default=1) or 1
    return 0


def stub_main(a, world, rank):
    """NLOSGR_BENCH_STUB=1: the launcher / barrier / timing path with a small CPU step (a
    [256,256] matmul per step + an all-reduce of a 64-float 'gradient', gloo) in place of the
    render.  Not a measurement: rehearses the contract without a GPU."""
    dev = torch.device("cpu")
    if world > 1:
        dist.init_process_group(os.environ.get("NLOSGR_DIST_BACKEND", "gloo"))
    if os.environ.get("NLOSGR_BENCH_STUB_FAIL_RANK") == str(rank):
        raise SystemExit(3)        # launcher test: a rank that dies after the rendezvous
    x = torch.randn(256, 256, generator=torch.Generator().manual_seed(rank))
    grad = torch.zeros(64)

    def step():
        t0 = time.perf_counter()
        y = x @ x
        grad.fill_(float(y[0, 0]))
        if world > 1:
            dist.all_reduce(grad)
        ms = (time.perf_counter() - t0) * 1e3
        return lambda: (ms, 0.0)

    elapsed, own, phases = timed_run(step, a.steps, a.warmup, world, dev)
    ranks = _gather_ranks(world, rank, own, phases, "cpu")
    if rank == 0:
        print(json.dumps({"metric": "stub (launcher rehearsal)", "value": world * 1000.0 * a.steps / (elapsed * 1e3),
                          "unit": "steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": elapsed * 1e3 / a.steps, "ranks": ranks,
                          "dist": _dist_info(world)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _dist_info(world):
    if world == 1 or not dist.is_initialized():
        return {"backend": None, "world_size": 1}
    return {"backend": str(dist.get_backend()), "world_size": dist.get_world_size()}


def _gather_ranks(world, rank, own, phases, device):
    """Every rank's own timed wall time and mean phase times, gathered on rank 0."""
    mine = {"rank": rank, "device": device, "ms_per_step": own * 1e3 / max(1, len(phases)),
            "fwd_ms": statistics.fmean(p[0] for p in phases) if phases else 0.0,
            "bwd_ms": statistics.fmean(p[1] for p in phases) if phases else 0.0}
    if world == 1:
        return [mine]
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    return allr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--cutoff", type=float, default=5.7,
                    help="Mahalanobis support radius; 5.7 = parity grade (SURVEY §8d), <= 0 = dense")
    ap.add_argument("--lines", default="",
                    help="comma-separated extra cutoffs timed the same way (reported under 'lines'); '' = none")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--preset", default="cuda", choices=("cuda", "torch"),
                    help="convention preset: cuda = the reference's CUDA path, torch = its torch path (SURVEY A.3)")
    ap.add_argument("--mode", default="noocl", choices=("noocl", "netf", "occl"),
                    help="noocl (configs/default.py:15 default), netf self-transmittance, or occl = path C's "
                         "shared-transmittance compositing (ray-tile engine)")
    ap.add_argument("--selection", default="support", choices=("support", "aabb"),
                    help="support = Mahalanobis cutoff; aabb = path C's 3-sigma box filter, 256 per ray")
    ap.add_argument("--band", type=int, default=0,
                    help="single GPU: time EVERY band of a BAND-way wall shard in turn (one rank's share each); "
                         "value = projected job rate 1 / max-over-bands step time (the all-reduce is not timed)")
    ap.add_argument("--replicas", action="store_true",
                    help="with N ranks: every rank renders a full volume of its own capture (weak scaling)")
    a = ap.parse_args()

    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        # no launcher: start the N ranks ourselves, before any torch.cuda call in this process
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"[bench] WORLD_SIZE={world} but --gpus {a.gpus}: refusing to report a {world}-rank run "
              f"as {a.gpus} GPUs", file=sys.stderr, flush=True)
        sys.exit(2)
    if os.environ.get("NLOSGR_BENCH_STUB") == "1":
        return stub_main(a, world, rank)
    # NLOSGR_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (rank -> GPU local % count); the
    # production path is RCCL ("nccl"), one GPU per rank
    ndev = max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local % ndev)
        dist.init_process_group(os.environ.get("NLOSGR_DIST_BACKEND", "nccl"))
    dev = torch.device("cuda", local % ndev)
    if a.band > 1 and world > 1:
        raise SystemExit("--band is a single-GPU projection; with N ranks the wall is sharded by default")

    from nlosgr import GaussianParams
    from nlosgr.distributed import wall_rows
    from nlosgr.model import features_flat
    from nlosgr.render import count_support, render_forward
    from nlosgr.train import TrainStep
    from nlosgr.volume import Scene, make_config

    ng, H, W, T, ns, fwd_only = CONFIGS[a.config]
    scene = Scene(H=H, W=W, T=T, ns=ns)
    model = GaussianParams.synthetic(ng, 3, preset=a.preset, device=dev, seed=0)
    sharded = world > 1 and not a.replicas
    walls_all = scene.walls(dev)
    # shards: whole wall rows, row-interleaved over the ranks (balanced work; wall_rows)
    if sharded:
        bands = [(rank, world)]
    elif a.band > 1:
        bands = [(r, a.band) for r in range(a.band)]
    else:
        bands = [(0, 1)]
    g = torch.Generator().manual_seed(1 + (0 if sharded else rank))
    target_all = (torch.rand(H * W, T, generator=g) * 1e-3).to(dev)   # measured volume, x gt_times=100 in the loss
    stream = torch.cuda.current_stream(dev)
    cutoffs = [a.cutoff] + [float(x) for x in a.lines.split(",") if x.strip()]
    results = {}
    for cut in cutoffs:
        cfg = make_config(model, scene, a.preset, a.mode, cutoff=cut, selection=a.selection)
        per_band = []
        for (b0, b1) in bands:      # (shard, of shards)
            whole = b1 == 1
            idx = wall_rows(H, W, b0, b1, device=dev)
            geo = scene.geometry(dev, a.preset, a.mode, walls=None if whole else walls_all[idx].contiguous())
            target = target_all[idx].contiguous()
            ev_fwd = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev_bwd = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            train = TrainStep(model, geo, cfg, target, gt_times=100.0,
                              nwall_total=H * W if (sharded or a.band > 1) else H * W * world,
                              events={"fwd": ev_fwd, "bwd": ev_bwd})
            snap = Snapshot(train)

            def step():
                snap.restore()
                if fwd_only:
                    params = [model._mu.detach(), model._scaling.detach(), model._rotation.detach(),
                              model._opacity.detach(), features_flat(model).detach().contiguous()]
                    ev_fwd[0].record(stream)
                    render_forward(*params, geo, cfg, True, False)
                    ev_fwd[1].record(stream)
                    return lambda: (ev_fwd[0].elapsed_time(ev_fwd[1]), 0.0)
                train()
                return train.phase_ms   # HIP events of the step's phases (occl: summed over its batches)

            elapsed, own, evs = timed_run(step, a.steps, a.warmup, world, dev)
            fwd_ms = [e[0] for e in evs]
            bwd_ms = [e[1] for e in evs] if not fwd_only else []
            snap.restore()
            params = [model._mu.detach(), model._scaling.detach(), model._rotation.detach(),
                      model._opacity.detach(), features_flat(model).detach().contiguous()]
            if a.selection == "aabb":
                pairs = rays = evals = None      # no support count for the box filter
            else:   # occl: the same (pair, ray, bin) support as noocl at this cutoff
                pairs, rays, evals = count_support(*params, geo, replace(cfg, mode="noocl") if a.mode == "occl" else cfg)
            per_band.append({"band": [b0, b1], "ms_per_step": elapsed * 1000.0 / a.steps,
                             "fwd_ms": statistics.fmean(fwd_ms), "bwd_ms": statistics.fmean(bwd_ms) if bwd_ms else 0.0,
                             "fwd_ms_all": fwd_ms, "bwd_ms_all": bwd_ms, "pairs": pairs, "rays": rays,
                             "evaluations": evals, "nwall": int(idx.numel()), "own_s": own, "phases": evs})
            del train, snap
            torch.cuda.empty_cache()
        results[cut] = per_band

    main_bands = results[a.cutoff]
    worst = max(main_bands, key=lambda b: b["ms_per_step"])
    ms_per_step = worst["ms_per_step"]
    if sharded:
        volumes_per_s = 1000.0 / ms_per_step
    elif a.band > 1:
        volumes_per_s = 1000.0 / ms_per_step          # projected: every band on its own GPU
    else:
        volumes_per_s = world * 1000.0 / ms_per_step

    # HBM roofline of the dominant phase: algorithmic bytes per launch / its average HIP-event
    # duration (params read + dL/dV read + grads written for the backward)
    pb = param_bytes(3)
    V = 4 * worst["nwall"] * T
    fwd_avg, bwd_avg = worst["fwd_ms"], worst["bwd_ms"]
    tiles = a.mode == "occl" or a.selection == "aabb"     # ray-tile engine (csrc/nlosgr_tiles.hip)
    if bwd_avg >= fwd_avg:
        dom, dom_ms, dom_bytes = "bwd", bwd_avg, 2 * ng * pb + V
    else:
        dom, dom_ms, dom_bytes = "fwd", fwd_avg, ng * pb + V
    kern = PHASE_KERNELS[("tiles_" + dom) if tiles else dom]
    wl = {"preset": a.preset, "mode": a.mode, "selection": a.selection}
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    single = a.band <= 1 and world == 1
    phase_tr, traffic_src = pmc_traffic(a.config, a.cutoff, tiles, **wl) if single else ({"fwd": None, "bwd": None}, None)
    traffic = phase_tr[dom]
    # compute-side figures: exact in-support evaluations of the (frozen) workload per second, and the
    # VALU issue utilisation from the committed SQ counter pass of this command
    # (SQ_INSTS_VALU x 2 cycles per wave64 instruction / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs); the 2
    # cycles: MI355X_MICROARCH.md:54,473; v_exp_f32 measured at 8.2 (scripts/drain_proto.hip), so a lower bound)
    ev = worst["evaluations"]
    valu = {"evaluations": ev, "pairs": worst["pairs"], "rays": worst["rays"],
            "evals_per_s_fwd": ev / (fwd_avg * 1e-3) if ev else None,
            "evals_per_s_bwd": ev / (bwd_avg * 1e-3) if (ev and bwd_avg) else None}
    sq, sq_src = committed_profile(a.config, "valu", a.cutoff, **wl) if single else (None, None)
    if sq:
        valu["valu_issue_util"] = sq.get("valu_issue_util")
        valu["source"] = sq_src
    out = {
        "metric": "transient volumes/sec (fwd+bwd), 100k Gaussians → 128×128×1024 ToF bins"
        if a.config == "C3" and (a.preset, a.mode, a.selection) == ("cuda", "noocl", "support")
        else f"transient volumes/sec ({'fwd' if fwd_only else 'fwd+bwd'}) {a.config}",
        "value": volumes_per_s, "unit": "volumes/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True,
        "scaling": "strong" if sharded else "weak", "vs_baseline": None,
        "dtype": "f32", "data": "synthetic (SURVEY §8d geometry, seeded random Gaussians and target)",
        "config": {"workload": f"{a.config}: {ng} Gaussians -> {H}x{W} wall x {T} bins, {ns}x{ns} angular "
                               f"samples, {a.preset} preset, {'no occlusion' if a.mode == 'noocl' else a.mode}"
                               f"{', path C AABB selection (256 per ray)' if a.selection == 'aabb' else ''}, "
                               f"{'dense (every sample)' if a.cutoff <= 0 else f'support cutoff {a.cutoff} sigma'}, "
                               f"{'fwd' if fwd_only else 'fwd+MSE+bwd (6 param grads)+Adam'}, frozen workload",
                   "gaussians": ng, "wall": [H, W], "bins": T, "angular": ns, "cutoff": a.cutoff,
                   "preset": a.preset, "mode": a.mode, "selection": a.selection,
                   "parallelism": (f"wall shard: {world} row-interleaved shards (rank r renders wall rows r, r+{world}, ...), "
                                   f"bucketed grad all-reduce"
                                   if sharded else
                                   f"all {a.band} shards of a {a.band}-way row-interleaved wall shard timed in turn on one GPU "
                                   f"(projected job rate = 1 / slowest band; all-reduce not timed)" if a.band > 1 else
                                   f"replicas x{world} (own capture each), grad all-reduce" if world > 1 else
                                   "single GPU")},
        "phase_ms": {"fwd": fwd_avg, "bwd": bwd_avg},
        "roofline": {"bound": "hbm", "kernel": f"nlosgr {dom} ({' + '.join(kern)})", "achieved": achieved,
                     "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "traffic_per_phase": {"fwd": phase_tr["fwd"], "bwd": phase_tr["bwd"],
                                           "unit": "HBM bytes per step (PMC FETCH_SIZE x2 + WRITE_SIZE)"},
                     "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_ms": dom_ms},
        "compute": valu,
    }
    if world > 1:
        out["ranks"] = _gather_ranks(world, rank, main_bands[0]["own_s"], main_bands[0]["phases"], str(dev))
        out["dist"] = _dist_info(world)
    if a.band > 1:
        out["bands"] = [{k: b[k] for k in ("band", "ms_per_step", "fwd_ms", "bwd_ms", "evaluations")}
                        for b in main_bands]
    lines = []
    for cut in cutoffs[1:]:
        b = max(results[cut], key=lambda x: x["ms_per_step"])
        lines.append({"cutoff": cut, "value": (1 if (sharded or a.band > 1) else world) * 1000.0 / b["ms_per_step"],
                      "ms_per_step": b["ms_per_step"], "phase_ms": {"fwd": b["fwd_ms"], "bwd": b["bwd_ms"]},
                      "evaluations": b["evaluations"]})
    if lines:
        out["lines"] = lines
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(a.config, a.cutoff, preset=a.preset, mode=a.mode)
        except Exception as e:  # report, never fake
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
        if a.config == "C3" and (a.preset, a.mode, a.selection) == ("cuda", "noocl", "support"):
            # BASELINE.json configs[0] (1k Gaussians -> 32x32x128 on the CPU, the reference's torch path:
            # torch preset, dense) timed in the same run, for the record beside the headline's baseline
            try:
                out["cpu_baseline_c1"] = cpu_baseline("C1", 0.0, preset="torch", mode="noocl")
            except Exception as e:
                out["cpu_baseline_c1"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
