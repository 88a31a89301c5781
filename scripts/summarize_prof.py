"""Summarise a prof_c3.sh run into profiles/: per-kernel stats (copied) and per-launch HBM traffic
from the FETCH_SIZE / WRITE_SIZE passes (FETCH_SIZE doubled: MI355X_MICROARCH.md §HBM, gfx950
reports half the bytes of wide reads; WRITE_SIZE taken as is).  FETCH/WRITE_SIZE are in KB.

    python scripts/summarize_prof.py gpurun_out/prof_c3 r01_c3
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return acc


def main(src, tag):
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = [f for f in os.listdir(src) if f.startswith("kt_") and f.endswith("kernel_stats.csv")]
    for f in stats:
        shutil.copy(os.path.join(src, f), os.path.join(out, f"{tag}_kernel_stats.csv"))
    fetch = per_kernel(os.path.join(src, "fetch_c3_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "write_c3_counter_collection.csv"), "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        if "rocclr" in k or "elementwise" in k.lower() or "at::" in k:
            continue
        fb = 2.0 * 1024 * sum(fetch.get(k, [0])) / max(1, len(fetch.get(k, [1])))
        wb = 1024 * sum(write.get(k, [0])) / max(1, len(write.get(k, [1])))
        res[k] = {"fetch_bytes_x2": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb,
                  "launches": max(len(fetch.get(k, [])), len(write.get(k, [])))}
    sq = os.path.join(src, "sq_c3_counter_collection.csv")
    if os.path.exists(sq):   # keep only this library's kernels
        with open(sq) as f, open(os.path.join(out, f"{tag}_sq_counters.csv"), "w", newline="") as g:
            rd = csv.DictReader(f)
            wr = csv.DictWriter(g, fieldnames=rd.fieldnames)
            wr.writeheader()
            for row in rd:
                if "anonymous namespace" in row["Kernel_Name"]:
                    wr.writerow(row)
    with open(os.path.join(out, f"{tag}_traffic.json"), "w") as f:
        json.dump({"source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of bench.py ({tag})",
                   "kernels": res}, f, indent=1)
    for k, v in res.items():
        print(f"{v['hbm_bytes_per_launch'] / 1e6:10.2f} MB  {k[:90]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
