#!/usr/bin/env python3
"""Register / spill / LDS summary of the kernels in a hipcc -S listing.
usage: kres.py <file.s> [name-substring]"""
import re
import sys

s = open(sys.argv[1]).read()
key = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.split(r"\n  - \.", s.split("amdhsa.kernels:")[-1]):
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    name = g("name")
    if key in name:
        print(f"{name[:60]:60s} sgpr {g('sgpr_count'):>4} sspill {g('sgpr_spill_count'):>3} vgpr {g('vgpr_count'):>4} "
              f"vspill {g('vgpr_spill_count'):>3} lds {g('group_segment_fixed_size'):>6} priv {g('private_segment_fixed_size')}")
