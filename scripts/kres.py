"""VGPR / scratch / LDS per kernel from a device-only .s (scripts/kernel_resources.sh output)."""
import re, sys
s = open(sys.argv[1] if len(sys.argv) > 1 else "/tmp/nlosgr_isa/nlosgr_volume.s").read()
pat = sys.argv[2] if len(sys.argv) > 2 else "."
for blk in s.split("  - .")[1:]:
    m = re.search(r"\.name:\s+(\S+)", blk)
    if not m or not re.search(pat, m.group(1)):
        continue
    g = lambda k: (re.search(rf"\.{k}:\s+(\d+)", blk) or [None, "?"])[1]
    print(m.group(1).replace("_ZN12_GLOBAL__N_1", ""), "vgpr", g("vgpr_count"), "agpr", g("agpr_count"),
          "spill", g("vgpr_spill_count"), "scratch", g("private_segment_fixed_size"), "lds", g("group_segment_fixed_size"))
