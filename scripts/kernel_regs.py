"""VGPR count and scratch bytes per kernel of a -save-temps device assembly (build.py --save-temps leaves
nlosgr_<file>-hip-amdgcn-amd-amdhsa-gfx950.s in csrc/).

    python scripts/kernel_regs.py nlos-gaussian-renderer_amd/csrc/nlosgr_volume-hip-amdgcn-amd-amdhsa-gfx950.s [filter]"""
import re, sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ''
for blk in re.finditer(r'\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel', s, re.S):
    name, body = blk.group(1), blk.group(2)
    if flt not in name:
        continue
    v = re.search(r'amdhsa_next_free_vgpr (\d+)', body).group(1)
    sc = re.search(r'amdhsa_private_segment_fixed_size (\d+)', body).group(1)
    lds = re.search(r'amdhsa_group_segment_fixed_size (\d+)', body).group(1)
    print(f'{name}  vgpr {v}  scratch {sc}  lds {lds}')
