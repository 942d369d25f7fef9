"""Dev helper: the memory-op / wait / branch skeleton of one kernel in a .s file
(usage: python tools/loop_waits.py file.s kernel-regex)."""
import re
import sys

s = open(sys.argv[1]).read()
n = [x for x in re.findall(r"^(_Z\w+):", s, re.M) if re.search(sys.argv[2], x)][0]
body = s[s.index(n + ":"):]
body = body[:body.index(".Lfunc_end")]
keep = ("s_waitcnt", "buffer_", "global_", "s_cbranch", "s_branch", "v_mfma", "ds_", "v_permlane", "scratch_")
cnt = 0
for line in body.splitlines():
    t = line.strip()
    if re.match(r"^\.LBB\w+:", t):
        print(f"   ({cnt} other)\n{t}")
        cnt = 0
    elif t.startswith(keep):
        if cnt:
            print(f"   ({cnt} other)")
            cnt = 0
        print("  ", t[:90])
    elif t and not t.startswith((".", ";")):
        cnt += 1
print(f"   ({cnt} other)")
