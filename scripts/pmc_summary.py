"""Summarise rocprofv3 --pmc passes (rocpd sqlite): per kernel (name filter), per counter, the
value per dispatch (averaged over dispatches) plus derived ratios for the query kernel.
usage: python scripts/pmc_summary.py <kernel-substring> db1 [db2 ...]"""
import sqlite3
import sys
from collections import defaultdict

pat = sys.argv[1]
vals = defaultdict(list)
meta = {}
for db in sys.argv[2:]:
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, sum(value), grid_size, workgroup_size, "
                     "lds_block_size, vgpr_count, sgpr_count, end - start from counters_collection "
                     "group by dispatch_id, counter_name").fetchall()
    for d, name, cn, v, gs, ws, lds, vg, sg, dur in rows:
        if pat not in name:
            continue
        vals[cn].append(v)
        meta = {"kernel": name[:100], "grid": gs, "wg": ws, "lds": lds, "vgpr": vg, "sgpr": sg}
print(meta)
avg = {k: sum(v) / len(v) for k, v in vals.items()}
for k in sorted(avg):
    print(f"{k:28s} {avg[k]:16.0f}  (dispatches {len(vals[k])})")
g = avg.get
if g("SQ_WAVE_CYCLES"):
    wc = g("SQ_WAVE_CYCLES")
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
              "SQ_WAIT_INST_LDS"):
        if g(k):
            print(f"  {k} / WAVE_CYCLES = {g(k) / wc:.3f}")
if g("SQ_INSTS_VALU") and g("SQ_WAVES"):
    print(f"  VALU insts per wave = {g('SQ_INSTS_VALU') / g('SQ_WAVES'):.0f}")
if g("SQ_INSTS_LDS") and g("SQ_WAVES"):
    print(f"  LDS insts per wave = {g('SQ_INSTS_LDS') / g('SQ_WAVES'):.0f}")
if g("SQ_INSTS_SALU") and g("SQ_WAVES"):
    print(f"  SALU insts per wave = {g('SQ_INSTS_SALU') / g('SQ_WAVES'):.0f}")
if g("SQ_LDS_BANK_CONFLICT") and g("SQ_LDS_IDX_ACTIVE"):
    print(f"  LDS bank conflict / LDS active = {g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.3f}")
