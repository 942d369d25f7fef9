"""Dev helper: instruction histogram + register counts of one kernel in a .s file."""
import re, sys
from collections import Counter
s = open(sys.argv[1]).read()
pat = sys.argv[2]
names = re.findall(r"^(_Z\w+):", s, re.M)
k = [n for n in names if re.search(pat, n)]
for n in k:
    body = s[s.index(n + ":"):]
    body = body[:body.index(".Lfunc_end")]
    ins = [l.strip().split()[0] for l in body.splitlines() if l.startswith("\t") and not l.strip().startswith((".", ";"))]
    c = Counter(ins)
    meta = s[s.index(".name:           " + n) - 3000: s.index(".name:           " + n) + 1200]
    regs = dict(re.findall(r"\.(sgpr_count|vgpr_count|agpr_count|private_segment_fixed_size|group_segment_fixed_size):\s+(\d+)", meta))
    print(n[:90], "ins", len(ins), regs)
    if len(sys.argv) > 3:
        print(c.most_common(int(sys.argv[3])))
        print("\n".join(l for l in body.splitlines() if "dpp" in l or "global_load" in l or "global_store" in l))
