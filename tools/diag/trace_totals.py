"""Per-kernel totals of the LAST `reps` bursts of a rocprofv3 kernel trace (a burst = dispatches separated by less than
`gap_us` of idle GPU time), averaged per burst: `python tools/diag/trace_totals.py <kernel_trace.csv> <reps> [gap_us]`
-- e.g. the kernels of one short-prompt prefill (tools/diag/prefill_small.py: each timed generate is one burst, the
host work between generates the gap)."""
import csv
import sys
from collections import defaultdict


def main(path, reps, gap_us=150.0):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    bursts, cur, prev_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if prev_end is not None and (s - prev_end) / 1e3 > gap_us and cur:
            bursts.append(cur)
            cur = []
        cur.append(r)
        prev_end = max(prev_end or e, e)
    if cur:
        bursts.append(cur)
    take = bursts[-reps:]
    tot, cnt = defaultdict(float), defaultdict(int)
    walls = []
    for b in take:
        walls.append((int(b[-1]["End_Timestamp"]) - int(b[0]["Start_Timestamp"])) / 1e3)
        for r in b:
            k = r["Kernel_Name"][:90]
            tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            cnt[k] += 1
    n = len(take)
    walls.sort()
    print(f"{len(bursts)} bursts, last {n} analysed: {sum(len(b) for b in take) / n:.1f} dispatches, kernel busy "
          f"{sum(tot.values()) / n:.1f} us, wall p50 {walls[n // 2]:.1f} us per burst")
    for k in sorted(tot, key=tot.get, reverse=True)[:25]:
        print(f"  {tot[k] / n:9.1f} us  {cnt[k] / n:6.1f} calls  {tot[k] / cnt[k]:7.2f} us/call  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), float(sys.argv[3]) if len(sys.argv) > 3 else 150.0)
