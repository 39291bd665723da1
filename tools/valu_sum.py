"""Per-kernel PMC totals (per launch) from a rocprofv3 counter CSV, with per-element rates.
usage: python tools/valu_sum.py CSV ELEMENTS_PER_LAUNCH"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
units = float(sys.argv[2]) if len(sys.argv) > 2 else None
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
meta = {}
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
    meta[k] = (r["VGPR_Count"], r["Scratch_Size"], r["LDS_Block_Size"])
for k, v in agg.items():
    n = len(disp[k])
    print(k, f"launches={n} vgpr/scratch/lds={meta[k]}")
    for c, x in sorted(v.items()):
        per = x / n
        extra = f"  per elem x64: {per * 64 / units:.1f}" if units and c.startswith("SQ_INSTS") else ""
        print(f"   {c:24s} {per:.4g}{extra}")
