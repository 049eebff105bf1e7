#!/usr/bin/env python3
"""Time the in-graph decode sampler (csrc/kernels/sample.hip sample_decode_kernel) on a B-row decode step
of a 128K vocabulary: the service-load mix (half the rows temperature 0.7 / top-p 0.95, half greedy) and
other parameter sets.  python tools/sample_bench.py [--B 512] [--V 128256]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np
import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.engine.sampling import SamplingParams


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--V", type=int, default=128256)
    ap.add_argument("--scale", type=float, default=1.3, help="std of the synthetic logits")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, V = a.B, a.V
    g = torch.Generator(device=dev).manual_seed(0)
    base = torch.randn(B, V, device=dev, generator=g) * a.scale
    logits = base.clone()
    HIST = 64
    sets = {
        "service (T 0.7, top-p 0.95; half greedy)": (SamplingParams(temperature=0.7, top_p=0.95), 0.5),
        "T 0.7, top-k 40, top-p 0.95 (all rows)": (SamplingParams(temperature=0.7, top_p=0.95, top_k=40), 1.0),
        "T 1.0, no truncation (all rows)": (SamplingParams(temperature=1.0), 1.0),
        "T 0.7, top-p 0.95, repeat 1.1 (all rows)": (SamplingParams(temperature=0.7, top_p=0.95, repeat_penalty=1.1), 1.0),
    }
    for name, (p, frac) in sets.items():
        raw = np.frombuffer(ops.sample_params_bytes(p), dtype=np.uint8)
        grd = np.frombuffer(ops.sample_params_bytes(), dtype=np.uint8)
        ns = int(round(frac * B))
        params = torch.from_numpy(np.stack([raw] * ns + [grd] * (B - ns))).to(dev)
        seeds = torch.arange(B, dtype=torch.int64, device=dev) + 1
        pos = torch.full((B,), 300, dtype=torch.int32, device=dev)
        ctx = pos + 1
        hist = torch.randint(0, V, (B, HIST), dtype=torch.int32, device=dev)
        nxt = torch.zeros(B, dtype=torch.int32, device=dev)
        ts = []
        for it in range(12):
            logits.copy_(base)
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            ops.sample_decode(logits, B, params, seeds, pos, ctx, hist, nxt)
            s1.record()
            s1.synchronize()
            if it >= 2:
                ts.append(s0.elapsed_time(s1) * 1e3)
        print(f"{name:48s} B={B}: {np.median(ts):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
