#!/usr/bin/env python3
"""Kernel-time breakdown of a time window of a rocprofv3 kernel trace (e.g. the service-load burst at the
end of a bench.py run): GPU busy share of the window's wall time and the top kernels.

    trace_window.py run_kernel_trace.csv --last-s 5.3 [--top 25]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("nls_gemv::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name).strip()[:100]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last-s", type=float, required=True, help="window = the last S seconds of kernel activity")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(a.trace))]
    rows.sort()
    t_end = max(e for _, e, _ in rows)
    t0 = t_end - int(a.last_s * 1e9)
    win = [(s, e, n) for s, e, n in rows if s >= t0]
    agg, cnt = defaultdict(float), defaultdict(int)
    busy = 0.0
    last = t0
    for s, e, n in win:                          # union of kernel intervals (kernels do not overlap on one queue)
        busy += max(0, e - max(s, last))
        last = max(last, e)
        agg[short(n)] += (e - s) / 1e3
        cnt[short(n)] += 1
    wall = (t_end - t0) / 1e3
    tot = sum(agg.values())
    print(f"window {wall / 1e3:.3f} s: GPU busy {busy / 1e6:.3f} s ({100 * busy / 1e3 / wall:.1f} %), "
          f"{len(win)} kernels, kernel time {tot / 1e3:.1f} ms")
    for n, us in sorted(agg.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"{us / 1e3:10.1f} ms {100 * us / tot:5.1f}%  calls {cnt[n]:7d}  {n}")


if __name__ == "__main__":
    main()
