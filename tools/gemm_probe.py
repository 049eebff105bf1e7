#!/usr/bin/env python3
"""Run ONE quantised GEMV/GEMM shape repeatedly (for rocprofv3 --pmc passes and quick timing).

    python tools/gemm_probe.py --shape gateup --M 256 [--cfg 1,8,2,1] [--iters 50] [--type Q4_K]
Prints the median time per launch and effective TFLOP/s / GB/s.
"""
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
from nats_llm_studio_amd.gguf.synth import SPECS


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--shape", default="gateup")
    ap.add_argument("--M", type=int, default=256)
    ap.add_argument("--cfg", default="")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--type", default="Q4_K")
    ap.add_argument("--dense", action="store_true", help="give the weight its f16 copy (mode 4 eligible)")
    ap.add_argument("--ldx-pad", type=int, default=0, help="activation row stride = K + this (elements)")
    args = ap.parse_args()
    spec = SPECS[args.model]
    d, hd = spec.d_model, spec.head_dim
    t = GGMLType[args.type]
    rows, K, epi = {
        "qkv": ((spec.n_head + 2 * spec.n_kv_head) * hd, d, "f32"),
        "o": (d, spec.n_head * hd, "add"),
        "gateup": (2 * spec.d_ff, d, "swiglu"),
        "down": (d, spec.d_ff, "add"),
        "lm_head": (spec.vocab, d, "f32"),
    }[args.shape]
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    w = ops.QWeight(Q.random_blocks(t, rows * K, 0.02, rng), t, rows, K, dev)
    if args.dense:
        w.expand_dense()
    segs = [ops.Seg(w, 0)]
    M = args.M
    x = (torch.randn(M, K + args.ldx_pad, device=dev) * 0.5).to(ops.ACT_DTYPE)[:, :K]
    ncol = rows // 2 if epi == "swiglu" else rows
    y = torch.zeros(M, ncol, dtype=ops.ACT_DTYPE if epi == "swiglu" else torch.float32, device=dev)
    kw = {}
    if args.cfg:
        mode, waves, rt, ks = (int(v) for v in args.cfg.split(","))
        kw = dict(mode=mode, waves=waves, rt=rt, ks=ks)
    ops.qgemv(segs, x, y, M, epi=epi, **kw)
    torch.cuda.synchronize()
    ts = []
    for _ in range(args.iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        ops.qgemv(segs, x, y, M, epi=epi, **kw)
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    us = sorted(ts)[len(ts) // 2]
    print(f"{args.shape} {args.type} rows={rows} K={K} M={M} cfg={kw or 'table'}: {us:.2f} us  "
          f"{2.0 * M * rows * K / us / 1e6:.1f} TFLOP/s  {w.nbytes / us / 1e3:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
