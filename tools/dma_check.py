#!/usr/bin/env python3
"""Mode-3 (LDS-DMA) GEMM: correctness vs fp32 torch and timing vs mode 2 on the Llama-3-8B shapes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.gguf import quants as Q
from nats_llm_studio_amd.gguf.constants import GGMLType

dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
ok = True
for t in (GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q5_K):
    rows, K = 264, 768
    raw = Q.random_blocks(t, rows * K, 0.05, rng)
    w = ops.QWeight(raw, t, rows, K, dev)
    Wd = ops.QWeight(raw, t, rows, K, "cpu").dense()
    for M in (65, 256, 300):
        for mt, ks in ((16, 1), (8, 1), (16, 3)):
            x = (torch.randn(M, K) * 0.5).to(ops.ACT_DTYPE)
            y = torch.zeros(M, rows, device=dev)
            ops.qgemv([ops.Seg(w)], x.to(dev), y, M, mode=3, waves=4, rt=mt, ks=ks)
            torch.cuda.synchronize()
            ref = x.float() @ Wd.t()
            err = (y.cpu() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
            good = err < 2e-2
            ok &= good
            print(f"{t.name} M={M} mt={mt} ks={ks} relerr={err:.2e} {'OK' if good else 'FAIL'}", flush=True)
print("CORRECT" if ok else "WRONG", flush=True)
if not ok:
    sys.exit(1)

shapes = {"qkv": (6144, 4096, "f32"), "o": (4096, 4096, "add"), "gateup": (28672, 4096, "swiglu"),
          "down": (4096, 14336, "add"), "lm_head": (128256, 4096, "f32")}
for name, (rows, K, epi) in shapes.items():
    t = GGMLType.Q6_K if name == "lm_head" else GGMLType.Q4_K
    w = ops.QWeight(Q.random_blocks(t, rows * K, 0.02, rng), t, rows, K, dev)
    M = 256
    x = (torch.randn(M, K, device=dev) * 0.5).to(ops.ACT_DTYPE)
    ncol = rows // 2 if epi == "swiglu" else rows
    y = torch.zeros(M, ncol, dtype=ops.ACT_DTYPE if epi == "swiglu" else torch.float32, device=dev)
    res = []
    cfgs = [(2, 8, 4, k) for k in (1, 2, 4, 8)] + [(3, 4, mt, k) for mt in (16, 8) for k in (1, 2, 3, 4, 6, 8)]
    for cfg in cfgs:
        mode, waves, rt, ks = cfg
        if ks > K // 512:
            continue
        kw = dict(mode=mode, waves=waves, rt=rt, ks=ks)
        ops.qgemv([ops.Seg(w)], x, y, M, epi=epi, **kw)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(10):
                ops.qgemv([ops.Seg(w)], x, y, M, epi=epi, **kw)
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) / 10 * 1e3)
        res.append((sorted(ts)[2], cfg))
    res.sort()
    print(f"{name:8s} M={M} " + " ".join(f"{c}:{u:.1f}" for u, c in res[:6]) +
          f" | best mode2 {min(u for u, c in res if c[0] == 2):.1f} best mode3 {min(u for u, c in res if c[0] == 3):.1f}"
          f" ({2.0 * M * rows * K / res[0][0] / 1e6:.0f} TF/s)", flush=True)
