"""Dev tool: per-basic-block instruction counts of one kernel in the compiled
gfx950 assembly written by tools/isa_counts.py (/tmp/zkmi_isa/<SRC>.s).
usage: isa_blocks.py [kernel-substring] [min-valu]"""
import collections
import os
import re
import sys

name = sys.argv[1] if len(sys.argv) > 1 else "k_acc_items_g1"
minv = int(sys.argv[2]) if len(sys.argv) > 2 else 0
s = open(f"/tmp/zkmi_isa/{os.environ.get('SRC', 'msm')}.s").read()
m = re.search(r"^(_Z[^\s:]*" + re.escape(name) + r"[^\s:]*):", s, re.M)
body = s[m.start():s.index("s_endpgm", m.start())]
cur = "entry"
blocks = collections.OrderedDict({cur: collections.Counter()})
loops = {}
for line in body.splitlines()[1:]:
    t = line.strip()
    mm = re.match(r"^(\.LBB\w+):(.*)", t)
    if mm:
        cur = mm.group(1)
        blocks[cur] = collections.Counter()
        loops[cur] = mm.group(2).strip()[:40]
        continue
    if not t or t.startswith((".", ";", "//")):
        continue
    blocks[cur][t.split()[0]] += 1
for b, c in blocks.items():
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    if valu < minv:
        continue
    movs = c["v_mov_b32_e32"] + c["v_mov_b64_e32"]
    print(f"{b:12s} valu {valu:5d} mad {c['v_mad_u64_u32']:5d} other {valu - c['v_mad_u64_u32']:4d} "
          f"mov {movs:3d} nop {c['s_nop']:4d}  {loops.get(b, '')}")
