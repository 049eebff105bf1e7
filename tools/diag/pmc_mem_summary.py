#!/usr/bin/env python3
"""Summarise the memory-side PMC passes of tools/gpu_calls/r06/gpu_r6ad.sh: per probe (qkv_m4, ...), the mean per
dispatch of every counter over the GEMM kernel's dispatches (the probe's last 5 launches), plus derived rates.

    python tools/diag/pmc_mem_summary.py gpurun_out/pmc_ad
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def load(d):
    """{probe: {counter: mean value per GEMM dispatch}} and the probe's timing line."""
    out, times = {}, {}
    for tf in sorted(glob.glob(os.path.join(d, "*.time"))):
        n = os.path.basename(tf)[:-5]
        times[n] = open(tf).read().strip().splitlines()[-1]
        vals = defaultdict(list)
        for f in glob.glob(os.path.join(d, f"{n}_p*", "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(dict)
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if not re.search(r"hgemm|hg10|qgemm9|q9", k):
                    continue
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
            for disp in per.values():
                for c, v in disp.items():
                    vals[c].append(v)
        out[n] = {c: sum(v) / len(v) for c, v in vals.items() if v}
    return out, times


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_ad"
    data, times = load(d)
    for n, c in data.items():
        print(f"== {n}: {times.get(n, '')}")
        for k in sorted(c):
            print(f"   {k:36s} {c[k]:.4g}")
        g = lambda k: c.get(k, float("nan"))
        hit = g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum"))
        cyc = g("GRBM_GUI_ACTIVE") / 8            # dispatch cycles (GRBM sums the 8 XCDs)
        print(f"   -> L2 hit rate {hit:.3f}; L2 misses to fabric {g('TCC_EA0_RDREQ_sum'):.4g} req "
              f"({g('TCC_EA0_RDREQ_DRAM_sum'):.4g} to DRAM)")
        print(f"   -> L1->L2 read requests {g('TCP_TCC_READ_REQ_sum'):.4g}, mean latency "
              f"{g('TCP_TCC_READ_REQ_LATENCY_sum') / max(g('TCP_TCC_READ_REQ_sum'), 1):.0f} cycles; "
              f"TLB miss rate {g('TCP_UTCL1_TRANSLATION_MISS_sum') / max(g('TCP_UTCL1_TRANSLATION_MISS_sum') + g('TCP_UTCL1_TRANSLATION_HIT_sum'), 1):.4f}")
        print(f"   -> per CU per dispatch cycle: TA busy {g('TA_TA_BUSY_sum') / 256 / cyc:.3f}, TA addr stalled by TC "
              f"{g('TA_ADDR_STALLED_BY_TC_CYCLES_sum') / 256 / cyc:.3f}, TD busy {g('TD_TD_BUSY_sum') / 256 / cyc:.3f}, "
              f"TD stalled by TC {g('TD_TC_STALL_sum') / 256 / cyc:.3f}, TCP pending stall "
              f"{g('TCP_PENDING_STALL_CYCLES_sum') / 256 / cyc:.3f}")
        print(f"   -> MFMA pipe utilisation {g('SQ_VALU_MFMA_BUSY_CYCLES') / (1024 * cyc):.3f} "
              f"(dispatch {cyc:.0f} cycles)")


if __name__ == "__main__":
    main()
