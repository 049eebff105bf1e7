#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/.../run_counter_collection.csv):
per kernel name, the counter totals of its LAST dispatch plus derived ratios."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
US = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0      # kernel time (us) of the probe, for the clock
SIMDS, XCDS = 256 * 4, 8
# SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles: their ratios to each other are exact
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
    if c.get("SQ_VALU_MFMA_BUSY_CYCLES") and c.get("GRBM_GUI_ACTIVE"):
        # SQ_VALU_MFMA_BUSY_CYCLES: shader cycles of MFMA issue summed over every SIMD (16 per 16x16x32, 32 per
        # 32x32x16 instruction); GRBM_GUI_ACTIVE: the dispatch's cycles summed over the 8 XCDs
        # (MI355X_MICROARCH.md 'Per-instruction cycle constants', 'DVFS give-back'). Utilisation = busy cycles /
        # (SIMDs x kernel cycles), i.e. the share of the matrix pipe's cycles that issued an MFMA.
        kcyc = c["GRBM_GUI_ACTIVE"] / XCDS
        print(f"   MFMA pipe utilisation {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (SIMDS * kcyc):.3f} "
              f"(MFMA busy cycles / ({SIMDS} SIMDs x {kcyc:.4g} kernel cycles)"
              + (f", effective clock {kcyc / US / 1e3:.2f} GHz" if US else "") + ")")
    if c.get("SQ_WAVE_CYCLES"):
        w = c["SQ_WAVE_CYCLES"]
        print(f"   of wave cycles: wait_any {c.get('SQ_WAIT_ANY',0)/w:.3f} wait_inst {c.get('SQ_WAIT_INST_ANY',0)/w:.3f} "
              f"active {c.get('SQ_ACTIVE_INST_ANY',0)/w:.3f} valu {c.get('SQ_ACTIVE_INST_VALU',0)/w:.3f} "
              f"lds {c.get('SQ_ACTIVE_INST_LDS',0)/w:.3f}")
