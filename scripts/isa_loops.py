"""Per-loop instruction mix of one kernel in a hipcc -S listing (static counts; spots SGPR-spill
v_readlane/v_writelane traffic inside hot loops).
usage: python scripts/isa_loops.py file.s <mangled-kernel-name-substring>"""
import re
import sys

s = open(sys.argv[1]).read()
i = s.index(sys.argv[2])
i = s.index(":\n", i)
j = s.index(".Lfunc_end", i)
body = s[i:j].split("\n")
labels = {}
for n, l in enumerate(body):
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        labels[m.group(1)] = n
loops = set()
for n, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", l)
    if m:
        t = m.group(1) or m.group(2)
        if t in labels and labels[t] < n:
            loops.add((labels[t], n))
pats = {"valu": r"^\s+v_", "lane_spill": r"v_readlane|v_writelane", "ds": r"^\s+ds_", "med3": r"v_med3",
        "salu": r"^\s+s_", "vmem": r"^\s+(global|buffer)_", "waitcnt": r"s_waitcnt"}
for a, b in sorted(loops):
    seg = body[a:b + 1]
    c = {k: sum(1 for x in seg if re.search(p, x)) for k, p in pats.items()}
    print(f"loop lines {a}-{b} ({b - a}): " + ", ".join(f"{k} {v}" for k, v in c.items()))
