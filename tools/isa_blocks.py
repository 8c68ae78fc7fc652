"""Instruction mix per basic block of the kernels in a hipcc --save-temps .s file (gfx950): for each
kernel matching the regex, the blocks with the most scalar instructions and whether they sit in a
loop (a later block branches back to them). usage: python3 tools/isa_blocks.py FILE.s REGEX [min_salu]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2])
min_salu = int(sys.argv[3]) if len(sys.argv) > 3 else 40
for m in re.finditer(r"^(_Z\w+):", s, re.M):
    name = m.group(1)
    if not pat.search(name):
        continue
    end = s.find(".Lfunc_end", m.end())
    body = s[m.end():end].splitlines()
    blocks, cur, lab, order = [], [], "entry", {}
    for ln in body:
        mm = re.match(r"^(\.LBB[\w_]+):", ln)
        if mm:
            blocks.append((lab, cur))
            lab, cur = mm.group(1), []
        else:
            t = ln.strip()
            if t and not t.startswith((".", ";")):
                cur.append(t)
    blocks.append((lab, cur))
    for i, (lab, _) in enumerate(blocks):
        order[lab] = i
    back = set()
    for i, (lab, ins) in enumerate(blocks):
        for t in ins:
            mm = re.match(r"s_cbranch_\w+\s+(\.LBB[\w_]+)|s_branch\s+(\.LBB[\w_]+)", t)
            if mm:
                tgt = mm.group(1) or mm.group(2)
                if tgt in order and order[tgt] <= i:
                    back.update(l for l, _ in blocks[order[tgt]:i + 1])
    hot = []
    for lab, ins in blocks:
        ops = [t.split()[0] for t in ins]
        c = collections.Counter(ops)
        salu = sum(v for k, v in c.items() if k.startswith("s_") and not k.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_cbranch", "s_branch", "s_setprio", "s_sleep")))
        if salu >= min_salu:
            hot.append((salu, lab, len(ops), lab in back))
    if hot:
        print(name[:90])
        for salu, lab, n, inloop in sorted(hot, reverse=True)[:6]:
            print(f"   {lab:14s} salu {salu:4d} of {n:4d}{'  (in a loop)' if inloop else ''}")
