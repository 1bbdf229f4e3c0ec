"""Register / LDS / spill census of every kernel in a gfx950 assembly file (hipcc -S).
usage: python scripts/isa_resources.py file.s [name-substring]"""
import re
import sys

txt = open(sys.argv[1]).read()
sub = sys.argv[2] if len(sys.argv) > 2 else ""
# the amdhsa metadata block lists one map per kernel: .name, .sgpr_count, .vgpr_count, ...
for blk in re.split(r"\n  - \.", txt.split("amdhsa.kernels:")[-1])[1:]:
    f = dict(re.findall(r"\.(\w+):\s+(\S+)", "." + blk))
    name = f.get("name", "?")
    if sub and sub not in name:
        continue
    print(f"{name[:90]:90s} vgpr {f.get('vgpr_count')} agpr {f.get('agpr_count')} sgpr {f.get('sgpr_count')} "
          f"vspill {f.get('vgpr_spill_count')} sspill {f.get('sgpr_spill_count')} lds {f.get('group_segment_fixed_size')} "
          f"scratch {f.get('private_segment_fixed_size')}")
