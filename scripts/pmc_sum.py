"""Sum rocprofv3 counter_collection.csv values per (kernel, counter) for the nlosgr kernels."""
import csv, sys
from collections import defaultdict
agg = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if "fwd_kernel" not in k and "bwd_kernel" not in k:
        continue
    name = ("fwd" if "fwd_kernel" in k else "bwd") + "<" + k.split("<")[1].split(">")[0] + ">"
    agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, " ".join(f"{c}={x:.4g}" for c, x in sorted(v.items())))
