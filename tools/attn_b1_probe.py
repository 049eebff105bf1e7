#!/usr/bin/env python3
"""Batch-1 decode attention latency in isolation (Llama-3-8B heads: 32 q / 8 kv, D = 128, 16-token blocks),
captured in a hipGraph: the attention launch alone, a trivial launch alone (the boundary floor), and the two
interleaved (attention after another kernel, as in a decode layer). Per-launch microseconds, one JSON line per
context length. The production split policy and chunk are used (models/llama.py attn_splits, _MIN_CHUNK).
    python tools/attn_b1_probe.py [--ctx 128,512,2048] [--kv bf16|fp8]
(NLS_ATTN_MFMA_WAVES=4|8 selects the workgroup size per process.)"""
import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.models import llama

REPS = 64


def timed(fn, iters=7):
    fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(REPS):
            fn(i)
    best = math.inf
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / REPS)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", default="128,512,2048")
    ap.add_argument("--kv", default="bf16")
    ap.add_argument("--splits", type=int, default=0, help="override the split count (0: the production policy)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    kvt = torch.bfloat16 if a.kv == "bf16" else torch.float8_e4m3fn
    Hq, Hkv, D, bs = 32, 8, 128, 16
    nblk = 4096
    kc = (torch.randn(nblk * bs, Hkv, D, device=dev) * 0.5).to(kvt)
    vc = (torch.randn(nblk * bs, Hkv, D, device=dev) * 0.5).to(kvt)
    q = torch.randn(1, Hq * D, device=dev).to(torch.bfloat16)
    out = torch.zeros(1, Hq * D, dtype=ops.ACT_DTYPE, device=dev)
    ts = torch.zeros(1, dtype=torch.int32, device=dev)
    dummy = torch.zeros(256, device=dev)
    ns = a.splits or llama.LlamaModel.attn_splits(1, Hkv)
    ws = torch.zeros(Hq * ns * (D + 2), dtype=torch.float32, device=dev)
    cnt = torch.zeros(Hkv, dtype=torch.int32, device=dev)
    for ctx in [int(c) for c in a.ctx.split(",")]:
        bt = torch.randperm(nblk, device=dev)[: (ctx + bs - 1) // bs].to(torch.int32).view(1, -1).contiguous()
        cl = torch.tensor([ctx], dtype=torch.int32, device=dev)

        def attn(i):
            ops.attention(q, kc, vc, bt, ts, cl, out, 1, Hq, Hkv, D, bs, D ** -0.5, chunk=-llama._MIN_CHUNK,
                          n_split=ns, workspace=ws, counters=cnt)

        def triv(i):
            dummy.add_(1.0)

        def both(i):
            triv(i)
            attn(i)
        t_attn, t_triv, t_both = timed(attn), timed(triv), timed(both)
        print(json.dumps(dict(ctx=ctx, kv=a.kv, n_split=ns, waves_env=os.environ.get("NLS_ATTN_MFMA_WAVES"),
                              mfma_env=os.environ.get("NLS_ATTN_MFMA"),
                              attn_us=round(t_attn, 2), trivial_us=round(t_triv, 2), pair_us=round(t_both, 2),
                              attn_after_kernel_us=round(t_both - t_triv, 2))), flush=True)


if __name__ == "__main__":
    main()
