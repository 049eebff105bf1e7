#!/usr/bin/env python3
"""Kernel trace of the tensor-parallel rehearsal (parallel/rehearsal.py under rocprofv3 --kernel-trace): per
rank (trace file / host thread), the kernels of one greedy decode step -- delimited by the vocab-parallel
arg-max (oneshot_argmax_kernel), the last kernel of a TP decode step -- and a whole-run count of RCCL kernels.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tp_prof -o %pid%_run -- \
        python3 -m nats_llm_studio_amd.parallel.rehearsal --no-ref --profile-steps 8
    python tools/tp_trace.py gpurun_out/tp_prof
"""
import csv
import glob
import os
import re
import sys
from collections import Counter, defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", n).strip()[:70]


def main():
    root = sys.argv[1]
    files = sorted(glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True))
    groups = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            groups[(os.path.basename(f), r.get("Thread_Id", ""))].append(r)
    rccl = Counter()
    for (f, tid), rows in sorted(groups.items()):
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        for r in rows:
            if re.search(r"nccl|rccl", r["Kernel_Name"], re.I):
                rccl[short(r["Kernel_Name"])] += 1
        steps, cur = [], []
        for r in rows:
            cur.append(r)
            if "oneshot_argmax_kernel" in r["Kernel_Name"]:
                steps.append(cur)
                cur = []
        if len(steps) < 3:
            continue
        step = steps[-2]
        t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
        print(f"== {f} thread {tid}: {len(rows)} kernels, {len(steps)} TP steps; one greedy decode step = "
              f"{len(step)} kernels, {(t1 - t0) / 1e3:.1f} us first start -> last end")
        c = Counter(short(r["Kernel_Name"]) for r in step)
        dur = Counter()
        for r in step:
            dur[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for k, n in c.most_common():
            print(f"   {n:4d} x {dur[k]:9.1f} us  {k}")
    print(f"RCCL/NCCL kernels in the whole trace: {sum(rccl.values())} {dict(rccl)}")


if __name__ == "__main__":
    main()
