#!/usr/bin/env python3
"""The Mixtral-8x7B grouped expert GEMMs of one decode step at T tokens (top-2 of 8, random routing, ~T/4 rows per
expert), timed per launch (median of hipGraph replays) for rocprofv3 --pmc passes and A/Bs of the launch config.

    python tools/diag/moe_probe.py --proj gateup --T 256 [--cfg 2,8,4,1] [--iters 20] [--type Q5_K]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np
import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.gguf import quants as Q
from nats_llm_studio_amd.gguf.constants import GGMLType


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proj", default="gateup", choices=("gateup", "down"))
    ap.add_argument("--T", type=int, default=256)
    ap.add_argument("--cfg", default="2,8,4,1")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--type", default="Q5_K")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    E, k, d, ff = 8, 2, 4096, 14336
    rows, K, epi = (2 * ff, d, "swiglu") if a.proj == "gateup" else (d, ff, "f32")
    t = GGMLType[a.type]
    rng = np.random.default_rng(0)
    raw = Q.random_blocks(t, rows * K, 0.02, rng)
    ws = [ops.QWeight(raw, t, rows, K, dev) for _ in range(E)]      # same values, separate copies (E x HBM)
    T = a.T
    cap = T * k
    sel = np.stack([rng.choice(E, k, replace=False) for _ in range(T)])
    xrows = np.zeros(E * cap, np.int32)
    yrows = np.zeros(E * cap, np.int32)
    cnt = np.zeros(E, np.int32)
    for tok in range(T):
        for s, e in enumerate(sel[tok]):
            xrows[e * cap + cnt[e]] = tok if a.proj == "gateup" else tok * k + s
            yrows[e * cap + cnt[e]] = tok * k + s
            cnt[e] += 1
    xr, yr, cn = (torch.from_numpy(v).to(dev) for v in (xrows, yrows, cnt))
    segs = [ops.Seg(w, 0, xr[e * cap:], yr[e * cap:], cn[e:e + 1]) for e, w in enumerate(ws)]
    nx = T if a.proj == "gateup" else T * k
    x = (torch.randn(nx, K, device=dev) * 0.5).to(ops.ACT_DTYPE)
    ncol = rows // 2 if epi == "swiglu" else rows
    y = torch.zeros(T * k, ncol, dtype=ops.ACT_DTYPE if epi == "swiglu" else torch.float32, device=dev)
    mode, waves, rt, ks = (int(v) for v in a.cfg.split(","))
    M = T if a.proj == "gateup" else T * k
    fn = lambda: ops.qgemv(segs, x, y, M, epi=epi, mode=mode, waves=waves, rt=rt, ks=ks)
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    ts = []
    for _ in range(a.iters):
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        g.replay()
        s1.record()
        s1.synchronize()
        ts.append(s0.elapsed_time(s1) * 1e3)
    us = sorted(ts)[len(ts) // 2]
    nbytes = sum(w.nbytes for w in ws)
    print(f"{a.proj} T={T} cfg={a.cfg} counts={cnt.tolist()} {us:.1f} us  {nbytes / us / 1e3:.0f} GB/s of expert weights "
          f"({nbytes / 1e6:.0f} MB)", flush=True)


if __name__ == "__main__":
    main()
