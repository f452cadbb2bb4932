"""Per-basic-block VALU counts of one kernel in build/nw_kernels.s (blocks
with at least --min VALU instructions).  python tools/asm_blocks.py <substr>"""
import re
import sys
from collections import Counter

sub = sys.argv[1]
mn = int(sys.argv[2]) if len(sys.argv) > 2 else 40
s = open("sequencealigning_amd/build/nw_kernels.s").read()
names = [m.group(1) for m in re.finditer(r"^(_Z\S+):", s, re.M) if sub in m.group(1)]
for name in names:
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    blocks, cur, lab = [], [], "entry"
    for l in s[i:j].split("\n"):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            blocks.append((lab, cur))
            lab, cur = m.group(1), []
        elif l.strip() and not l.strip().startswith((";", ".", "/")):
            cur.append(l.strip().split()[0])
    blocks.append((lab, cur))
    print(name)
    for lab, ins in blocks:
        c = Counter(ins)
        v = sum(n for k, n in c.items() if k.startswith("v_"))
        if v >= mn:
            print(f"  {lab}: valu={v} total={len(ins)}",
                  sorted(((k, n) for k, n in c.items() if n > 2), key=lambda x: -x[1])[:12])
