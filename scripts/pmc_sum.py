"""Sum rocprofv3 counter_collection.csv values per (kernel, counter) for the nlosgr kernels."""
import csv, re, sys
from collections import defaultdict
agg = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if "fwd_" not in k and "bwd_" not in k and "tile_kernel" not in k:
        continue
    mt = re.search(r"(\w+_kernel)(<[^>]*>)?", k)
    name = mt.group(1) + (mt.group(2) or "") if mt else k
    agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, " ".join(f"{c}={x:.4g}" for c, x in sorted(v.items())))
