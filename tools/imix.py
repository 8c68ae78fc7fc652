"""Static instruction mix of one kernel in a hipcc device-asm file (straight-line kernels: static
counts ≈ per-wave dynamic counts). usage: python tools/imix.py FILE.s SUBSTR [top]
Build the asm with: hipcc -O3 -std=c++17 -fno-slp-vectorize -Iinclude -Ispwgnn_amd/csrc
  --offload-arch=gfx950 -x hip --cuda-device-only -S spwgnn_amd/csrc/kernels_fwd.hip -o /tmp/f.s"""
import collections
import re
import sys

txt = open(sys.argv[1]).read().split("\n")
sub = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
body, on = [], False
for ln in txt:
    m = re.match(r"^(_Z\S+):", ln)
    if m:
        on = sub in m.group(1) and not on
        if on:
            print("kernel", m.group(1)[:120])
        continue
    if on:
        if ln.strip().startswith(".Lfunc_end"):
            break
        s = ln.strip()
        if s and not s.startswith((".", ";")) and not s.endswith(":"):
            body.append(s.split()[0])
cnt = collections.Counter(body)
cls = collections.Counter()
for op, n in cnt.items():
    if op.startswith("v_mfma"):
        cls["mfma"] += n
    elif op.startswith(("v_", )):
        cls["valu"] += n
    elif op.startswith(("global_", "buffer_")):
        cls["vmem"] += n
    elif op.startswith("ds_"):
        cls["lds"] += n
    elif op.startswith("s_"):
        cls["salu/ctl"] += n
    else:
        cls["other"] += n
print(dict(cls), "total", sum(cls.values()))
for op, n in cnt.most_common(top):
    print(f"{n:7d} {op}")
