"""Summarise a prof_c3.sh run into profiles/ (all per launch, averaged over the run's launches):
  <tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  <tag>_traffic.json       HBM bytes = FETCH_SIZE x2 + WRITE_SIZE (MI355X_MICROARCH.md §HBM: gfx950
                           reports half the bytes of wide reads; WRITE_SIZE as is; both in KB)
  <tag>_valu.json          SQ + GRBM pass: VALU issue utilisation = SQ_INSTS_VALU x 2 cycles per
                           wave64 instruction / (128 SIMDs per XCD x GRBM_GUI_ACTIVE), GRBM_GUI_ACTIVE
                           being the sum over the 8 XCDs of each XCD's busy cycles (so 1024 SIMDs x
                           GRBM/8).  The 2 cycles: MI355X_MICROARCH.md:54 ("issues each VALU
                           instruction over 2 cycles (32 lanes/cycle x 2)") and :473 (v_fma_f32 wave64
                           2 cyc on SIMD-32); measured here 2.6 for a v_fma_f32 chain incl. loop
                           overhead, and 8.2 for v_exp_f32 (scripts/drain_proto.hip V0).  Every
                           transcendental therefore issues 4x longer than this counts: a lower bound.
  <tag>_sq_counters.csv    the raw SQ/GRBM rows of this library's kernels (LDS pass counters merged
                           into <tag>_valu.json per kernel)
  <tag>_bench.json         the bench line of the same command, its roofline.traffic and VALU figure
                           restated from this run's passes

    python scripts/summarize_prof.py gpurun_out/prof_c3 r02_c3
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path):
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def ours(k):
    return "anonymous namespace" in k or "nlosgr" in k


def short(k):
    return k.replace("(anonymous namespace)::", "").replace("nlosgr::detail::", "").split("(")[0]


def main(src, tag):
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    bench = open(os.path.join(src, "bench_default.log")).read().strip().splitlines()[-1]
    line = json.loads(bench)
    cutoff = line["config"]["cutoff"]
    # the workload the committed records belong to (bench.py matches on all four keys)
    wl = {"cutoff": cutoff, "preset": line["config"].get("preset", "cuda"), "mode": line["config"].get("mode", "noocl"),
          "selection": line["config"].get("selection", "support")}
    nsteps = line["steps"] + line["warmup"]
    for f in glob.glob(os.path.join(src, "kt_*kernel_stats.csv")):
        shutil.copy(f, os.path.join(out, f"{tag}_kernel_stats.csv"))
    fetch = per_kernel(glob.glob(os.path.join(src, "fetch_*counter_collection.csv"))[0])
    write = per_kernel(glob.glob(os.path.join(src, "write_*counter_collection.csv"))[0])
    res = {}
    for k in sorted(set(fetch) | set(write)):
        if not ours(k):
            continue
        fl, wr_ = fetch.get(k, {}).get("FETCH_SIZE", []), write.get(k, {}).get("WRITE_SIZE", [])
        fb = 2.0 * 1024 * sum(fl) / max(1, len(fl))
        wb = 1024 * sum(wr_) / max(1, len(wr_))
        n = max(len(fl), len(wr_))
        # per step: the backward runs one bwd_kernel / sh_kernel launch per wall-point batch
        res[short(k)] = {"fetch_bytes_x2": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb,
                         "launches": n, "launches_per_step": n / nsteps, "hbm_bytes_per_step": (fb + wb) * n / nsteps}
    with open(os.path.join(out, f"{tag}_traffic.json"), "w") as f:
        json.dump({"source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of bench.py ({tag})",
                   **wl, "kernels": res}, f, indent=1)
    # the bench line read the previously committed traffic/VALU profiles when it ran: restate its
    # roofline.traffic from the passes of this same run
    sys.path.insert(0, ROOT)
    from bench import phase_traffic
    tiles = wl["mode"] == "occl" or wl["selection"] == "aabb"
    dom = line["roofline"]["kernel"].split()[1]          # "nlosgr fwd (...)" / "nlosgr bwd (...)"
    per = {ph: phase_traffic(res, ("tiles_" + ph) if tiles else ph)[0] for ph in ("fwd", "bwd")}
    if per.get(dom) is not None:
        line["roofline"]["traffic"] = per[dom]
        line["roofline"]["traffic_per_phase"] = {"fwd": per["fwd"], "bwd": per["bwd"],
                                                 "unit": "HBM bytes per step (PMC FETCH_SIZE x2 + WRITE_SIZE)"}
        line["roofline"]["traffic_source"] = f"profiles/{tag}_traffic.json"
    sqf = glob.glob(os.path.join(src, "sq_*counter_collection.csv"))
    if sqf:
        sq = per_kernel(sqf[0])
        for f in glob.glob(os.path.join(src, "lds_*counter_collection.csv")):   # LDS pass, merged per kernel
            for kname, c in per_kernel(f).items():
                for n, v in c.items():
                    sq[kname].setdefault(n, v)
        kern = {}
        for k, c in sq.items():
            if not ours(k):
                continue
            avg = {n: sum(v) / len(v) for n, v in c.items()}
            g = avg.get("GRBM_GUI_ACTIVE", 0.0)
            avg["valu_issue_util"] = 2.0 * avg.get("SQ_INSTS_VALU", 0.0) / (128.0 * g) if g else None
            avg["launches"] = max(len(v) for v in c.values())
            kern[short(k)] = avg
        dom = max((v for k, v in kern.items() if "fwd_kernel" in k or "bwd_kernel" in k or "tile_kernel" in k),
                  key=lambda v: v.get("GRBM_GUI_ACTIVE", 0.0) * v["launches"], default=None)   # busiest over the run
        with open(os.path.join(out, f"{tag}_valu.json"), "w") as f:
            json.dump({"source": f"rocprofv3 --pmc SQ_* GRBM_GUI_ACTIVE pass of bench.py ({tag})",
                       **wl, "formula": "2 * SQ_INSTS_VALU / (128 * GRBM_GUI_ACTIVE)",
                       "valu_issue_util": dom["valu_issue_util"] if dom else None, "kernels": kern}, f, indent=1)
        with open(sqf[0]) as f, open(os.path.join(out, f"{tag}_sq_counters.csv"), "w", newline="") as g:
            rd = csv.DictReader(f)
            wr = csv.DictWriter(g, fieldnames=rd.fieldnames)
            wr.writeheader()
            for row in rd:
                if ours(row["Kernel_Name"]):
                    wr.writerow(row)
        if dom and isinstance(line.get("compute"), dict):
            line["compute"]["valu_issue_util"] = dom["valu_issue_util"]
            line["compute"]["source"] = f"profiles/{tag}_valu.json"
    with open(os.path.join(out, f"{tag}_bench.json"), "w") as f:
        f.write(json.dumps(line) + "\n")
    for k, v in res.items():
        print(f"{v['hbm_bytes_per_step'] / 1e6:10.2f} MB/step ({v['launches_per_step']:.2f} launches)  {k[:90]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
