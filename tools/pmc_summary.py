#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/.../run_counter_collection.csv):
per kernel name, the counter totals of its LAST dispatch plus derived ratios."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = defaultdict(dict)
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    rows = list(csv.DictReader(open(f)))
    last = {}
    for r in rows:
        k = r["Kernel_Name"][:70]
        last.setdefault(k, {})
        did = int(r["Dispatch_Id"])
        last[k].setdefault(did, defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in last.items():
        did = max(d)
        vals[k].update(d[did])
for k, c in vals.items():
    if "qmm" not in k and "qgemv" not in k and "hgemm" not in k and len(vals) > 1:
        continue
    print(k)
    for n in sorted(c):
        print(f"   {n:28s} {c[n]:.4g}")
    m = c.get("SQ_INSTS_MFMA", 0)
    if m:
        print(f"   VALU/MFMA {c.get('SQ_INSTS_VALU',0)/m:.2f}  LDS/MFMA {c.get('SQ_INSTS_LDS',0)/m:.2f}")
    if c.get("SQ_BUSY_CYCLES"):
        print(f"   MFMA busy {c.get('SQ_VALU_MFMA_BUSY_CYCLES',0)/c['SQ_BUSY_CYCLES']/4:.3f} (per-SIMD est)")
    if c.get("SQ_WAVE_CYCLES"):
        w = c["SQ_WAVE_CYCLES"]
        print(f"   wait_any {c.get('SQ_WAIT_ANY',0)/w:.3f} wait_inst {c.get('SQ_WAIT_INST_ANY',0)/w:.3f} active {c.get('SQ_ACTIVE_INST_ANY',0)/w:.3f}"
              f"  valu {c.get('SQ_ACTIVE_INST_VALU',0)/w:.3f} mfma {c.get('SQ_ACTIVE_INST_MFMA',0)/w:.3f} lds {c.get('SQ_ACTIVE_INST_LDS',0)/w:.3f}")
