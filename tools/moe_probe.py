#!/usr/bin/env python3
"""Run ONE grouped MoE expert GEMM (mapped rows, every expert in one launch) repeatedly, for
rocprofv3 --pmc passes and quick timing:

    python tools/moe_probe.py --proj gateup --T 256 [--rt 4] [--mode 2] [--iters 30] [--type Q5_K]

Mixtral-8x7B shapes by default (8 experts, top-2, d 4096, d_ff 14336); the route comes from random
logits (uniform load, like the random-init bench model). Prints the median time per launch, the
expert-weight bytes streamed per second and the useful (unpadded) TFLOP/s."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
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
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--E", type=int, default=8)
    ap.add_argument("--d", type=int, default=4096)
    ap.add_argument("--ff", type=int, default=14336)
    ap.add_argument("--type", default="Q5_K")
    ap.add_argument("--mode", type=int, default=2)
    ap.add_argument("--waves", type=int, default=8)
    ap.add_argument("--rt", type=int, default=4)
    ap.add_argument("--ks", type=int, default=1)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    t = GGMLType[args.type]
    T, k, E = args.T, args.k, args.E
    rows, K = (2 * args.ff, args.d) if args.proj == "gateup" else (args.d, args.ff)
    raw = Q.random_blocks(t, rows * K, 0.02, np.random.default_rng(0))
    ws = [ops.QWeight(raw, t, rows, K, dev) for _ in range(E)]     # distinct copies in HBM
    if args.mode >= 4:
        for w in ws:
            w.expand_dense()
    cap = T
    logits = torch.randn(T, E, device=dev)
    topw = torch.zeros(T * k, device=dev)
    counts = torch.zeros(E, dtype=torch.int32, device=dev)
    xrows = torch.zeros(E * cap, dtype=torch.int32, device=dev)
    yrows = torch.zeros(E * cap, dtype=torch.int32, device=dev)
    ops.moe_route(logits, T, k, topw, counts, xrows, yrows, cap)
    if args.proj == "gateup":
        x = (torch.randn(T, K, device=dev) * 0.5).to(ops.ACT_DTYPE)
        y = torch.zeros(T * k, rows // 2, dtype=ops.ACT_DTYPE, device=dev)
        segs = [ops.Seg(ws[e], 0, xrows[e * cap:], yrows[e * cap:], counts[e:e + 1]) for e in range(E)]
        M, epi = T, "swiglu"
    else:
        x = (torch.randn(T * k, K, device=dev) * 0.5).to(ops.ACT_DTYPE)
        y = torch.zeros(T * k, rows, device=dev)
        segs = [ops.Seg(ws[e], 0, yrows[e * cap:], yrows[e * cap:], counts[e:e + 1]) for e in range(E)]
        M, epi = (T * k if args.ks > 1 else T), "f32"
    kw = dict(mode=args.mode, waves=args.waves, rt=args.rt, ks=args.ks)

    def launch():
        for s0 in range(0, E, 8):
            ops.qgemv(segs[s0:s0 + 8], x, y, M, epi=epi, **kw)
    launch()
    torch.cuda.synchronize()
    ts = []
    for _ in range(args.iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        launch()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    us = sorted(ts)[len(ts) // 2]
    wbytes = sum(w.nbytes for w in ws) if args.mode < 4 else sum(w.dense_bytes for w in ws)
    print(f"moe {args.proj} {args.type} E={E} T={T} k={k} rows={rows} K={K} counts={counts.tolist()} cfg={kw}: "
          f"{us:.2f} us  {wbytes / us / 1e3:.1f} GB/s  {2.0 * T * k * rows * K / us / 1e6:.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
