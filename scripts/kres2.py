"""VGPR / spill / LDS per kernel from the device assembly metadata (scripts/kernel_resources.sh output)."""
import re, sys
txt = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.split(r"\n\s+- \.agpr_count:", txt)[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or pat not in name.group(1):
        continue
    g = lambda k: (re.search(rf"\.{k}:\s+(\S+)", blk) or [None, "?"])[1]
    print(name.group(1)[-40:], "vgpr", g("vgpr_count"), "spill", g("vgpr_spill_count"), "lds", g("group_segment_fixed_size"),
          "scratch", g("private_segment_fixed_size"))
