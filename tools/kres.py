"""Per-kernel register / spill / occupancy summary from a hipcc -Rpass-analysis=kernel-resource-usage log.
usage: python3 tools/kres.py LOG [name-regex]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
cur, vals = None, {}
for line in s.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        if cur and (not pat or pat.search(cur)):
            print(f"{cur[:80]:80s} V {vals.get('VGPRs')} A {vals.get('AGPRs')} spill {vals.get('VGPRs Spill')} occ {vals.get('Occupancy [waves/SIMD]')} lds {vals.get('LDS Size [bytes/block]')}")
        cur, vals = m.group(1), {}
        continue
    m = re.search(r"remark:\s+([^:]+): (\S+) \[", line)
    if m and cur:
        vals[m.group(1).strip()] = m.group(2)
if cur and (not pat or pat.search(cur)):
    print(f"{cur[:80]:80s} V {vals.get('VGPRs')} A {vals.get('AGPRs')} spill {vals.get('VGPRs Spill')} occ {vals.get('Occupancy [waves/SIMD]')} lds {vals.get('LDS Size [bytes/block]')}")
