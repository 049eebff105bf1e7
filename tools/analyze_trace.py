#!/usr/bin/env python3
"""Per-step breakdown of a rocprofv3 kernel trace of bench.py: decode steps are delimited by the
argmax_unpack kernel that ends every forward; reports GPU busy vs wall per step and the kernel
mix of the last N decode steps.  usage: analyze_trace.py run_kernel_trace.csv|run_results.db [--last 20]"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("nls_gemv::", "").replace("void ", "")
    name = re.sub(r"\(.*", "", name)
    return name.strip()[:90]


def load_rows(path):
    """kernel_trace.csv (--output-format csv) or the rocpd sqlite .db (ROCm 7.2 default)."""
    if path.endswith(".db"):
        import sqlite3
        c = sqlite3.connect(path)
        return [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
                for n, s, e in c.execute("select name, start, end from kernels")]
    return list(csv.DictReader(open(path)))


def main():
    path = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 20
    rows = sorted(load_rows(path), key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], []
    for r in rows:
        cur.append(r)
        if "argmax_unpack" in r["Kernel_Name"]:
            steps.append(cur)
            cur = []
    # decode steps: those whose big GEMMs have grid of the decode bucket (skip prefill: has attn_prefill)
    dec = [s for s in steps if not any("attn_prefill" in r["Kernel_Name"] for r in s)]
    dec = dec[-last:]
    agg = defaultdict(float)
    cnt = defaultdict(int)
    walls, busys = [], []
    prev_end = None
    gaps = []
    for s in dec:
        t0 = int(s[0]["Start_Timestamp"])
        t1 = int(s[-1]["End_Timestamp"])
        walls.append((t1 - t0) / 1e3)
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s) / 1e3
        busys.append(busy)
        if prev_end is not None:
            gaps.append((t0 - prev_end) / 1e3)
        prev_end = t1
        for r in s:
            k = short(r["Kernel_Name"])
            agg[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            cnt[k] += 1
    n = max(1, len(dec))
    print(f"decode steps analysed: {len(dec)}  kernels/step: {sum(len(s) for s in dec) / n:.0f}")
    print(f"per step: wall(first start->last end) {sum(walls) / n:.1f} us, kernel busy {sum(busys) / n:.1f} us, "
          f"inter-step gap {sum(gaps) / max(1, len(gaps)):.1f} us")
    tot = sum(agg.values())
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:20]:
        print(f"  {v / n:9.1f} us/step {100 * v / tot:5.1f}%  calls/step {cnt[k] / n:5.1f}  {k}")


if __name__ == "__main__":
    main()
