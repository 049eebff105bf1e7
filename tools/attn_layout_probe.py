#!/usr/bin/env python3
"""Decode attention at a service-load shape (B rows x ctx keys, Llama-3-8B heads) in the current K/V layout
[slot][Hkv][D] vs a head-major emulation (one [slot][1][D] cache per kv head, one launch per head: each
head's keys of a block contiguous). Reports us per layer-call and the K/V bytes rate.
    python tools/attn_layout_probe.py [--B 512] [--ctx 256] [--perm]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np
import torch

from nats_llm_studio_amd import ops


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    for _ in range(reps):
        fn()
    s1.record()
    s1.synchronize()
    return s0.elapsed_time(s1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--ctx", type=int, default=256)
    ap.add_argument("--perm", action="store_true", help="random block placement (a churned pool)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, ctx, bs, Hq, Hkv, D = a.B, a.ctx, 16, 32, 8, 128
    nbr = (ctx + bs - 1) // bs
    nblk = B * nbr + 8
    order = torch.randperm(nblk)[: B * nbr] if a.perm else torch.arange(B * nbr)
    bt = order.view(B, nbr).to(torch.int32).to(dev)
    ts = torch.arange(B, dtype=torch.int32, device=dev)
    cl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
    q = torch.randn(B, Hq * D, device=dev).to(torch.bfloat16)
    out = torch.zeros(B, Hq * D, dtype=ops.ACT_DTYPE, device=dev)
    kc = torch.randn(nblk * bs, Hkv, D, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    nbytes = 2 * B * ctx * Hkv * D * 2
    t = timed(lambda: ops.attention(q, kc, vc, bt, ts, cl, out, B, Hq, Hkv, D, bs, 0.088, chunk=-64))
    print(f"[slot][Hkv][D]          B={B} ctx={ctx}: {t:8.1f} us  {nbytes / t / 1e6:6.2f} TB/s", flush=True)
    ref = out.clone()
    G = Hq // Hkv
    kh = [kc[:, h:h + 1].contiguous() for h in range(Hkv)]
    vh = [vc[:, h:h + 1].contiguous() for h in range(Hkv)]
    outs = torch.zeros_like(out)

    def per_head():
        for h in range(Hkv):
            ops.attention(q[:, h * G * D:], kh[h], vh[h], bt, ts, cl, outs[:, h * G * D:], B, G, 1, D, bs, 0.088,
                          chunk=-64)
    t2 = timed(per_head)
    err = (outs.float() - ref.float()).abs().max().item()
    print(f"head-major (8 launches) B={B} ctx={ctx}: {t2:8.1f} us  {nbytes / t2 / 1e6:6.2f} TB/s  (max diff {err:.2e})",
          flush=True)


if __name__ == "__main__":
    main()
