"""Per-kernel register use from hipcc -S output (AMDGPU metadata): name, vgpr, agpr, spills.
usage: python tools/kres.py FILE.s [substr]"""
import re, sys
txt = open(sys.argv[1]).read()
sub = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.split(r"\n\s*- \.agpr_count:", txt)[1:]:
    agpr = int(blk.split("\n", 1)[0].strip())
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if name.endswith(".kd") or sub not in name:
        continue
    g = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", blk).group(1))
    print(f"{name[:70]:70s} vgpr={g('vgpr_count'):4d} agpr={agpr:4d} vspill={g('vgpr_spill_count'):3d} sspill={g('sgpr_spill_count'):3d}")
