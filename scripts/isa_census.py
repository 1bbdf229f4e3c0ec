"""Instruction census of one kernel in a gfx950 assembly file (hipcc --cuda-device-only -S):
total instructions, SGPR-spill traffic (v_writelane / v_readlane), and per-loop counts (each
backward branch target = a loop header; instructions between header and branch).
usage: python scripts/isa_census.py file.s kernel-substring"""
import re
import sys
from collections import Counter

txt = open(sys.argv[1]).read()
sub = sys.argv[2]
m = re.search(r"^(_Z\S*" + re.escape(sub) + r"\S*):", txt, re.M)
name = m.group(1)
start = m.end()
end = txt.index(".Lfunc_end", start)
lines = txt[start:end].splitlines()
ins = []  # (label or None, mnemonic, text)
labels = {}
for l in lines:
    if re.match(r"^\.LBB\S+:", l):
        labels[l.split(":")[0]] = len(ins)
        continue
    t = l.strip()
    if not t or t.startswith((".", ";")) or ":" in t.split()[0]:
        continue
    ins.append(t)
c = Counter(i.split()[0].replace("_e32", "").replace("_e64", "") for i in ins)
print(name[:100])
print("instructions", len(ins))
for k in ("v_readlane_b32", "v_writelane_b32", "v_med3_u32", "v_bfi_b32", "v_fma_f32", "v_sub_f32", "ds_read_b128",
          "v_cndmask_b32", "v_mov_b32", "v_readfirstlane_b32", "s_waitcnt", "scratch_load_dword", "scratch_store_dword"):
    print(f"  {k:22s} {c.get(k, 0)}")
# loops: backward branches
loops = []
for idx, t in enumerate(ins):
    if t.startswith("s_cbranch") or t.startswith("s_branch"):
        tgt = t.split()[-1]
        if tgt in labels and labels[tgt] <= idx:
            body = ins[labels[tgt]:idx + 1]
            cc = Counter(b.split()[0].replace("_e32", "").replace("_e64", "") for b in body)
            loops.append((labels[tgt], idx, len(body), cc.get("v_readlane_b32", 0), cc.get("v_writelane_b32", 0),
                          cc.get("v_med3_u32", 0), cc.get("v_mov_b32", 0), sum(v for k, v in cc.items() if k.startswith("v_"))))
print("loops (start, end, instrs, readlane, writelane, med3, mov, valu):")
for lp in sorted(loops):
    print("  ", lp)
