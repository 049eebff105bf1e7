#!/usr/bin/env python3
"""hipBLASLt f16 GEMM (torch.mm, f32 output) on the Llama-3-8B projection shapes at decode batch M:
the ceiling of a pre-dequantised (f16 weight copy) large-batch path, to compare with the quantised kernels."""
import sys

import torch

M = int(sys.argv[1]) if len(sys.argv) > 1 else 256
dev = torch.device("cuda:0")
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gateup": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}
for name, (N, K) in shapes.items():
    w = (torch.randn(N, K, device=dev) * 0.02).half()
    x = torch.randn(M, K, device=dev).half()
    out = {}
    for tag, fn in (("f16out", lambda: torch.mm(x, w.t())),
                    ("f32out", lambda: torch.mm(x, w.t(), out_dtype=torch.float32))):
        try:
            fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(10):
                    fn()
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
            out[tag] = sorted(ts)[2]
        except Exception as ex:
            out[tag] = f"err {str(ex)[:80]}"
    us = out.get("f32out") if isinstance(out.get("f32out"), float) else out.get("f16out")
    tf = 2.0 * M * N * K / us / 1e6 if isinstance(us, float) else 0
    print(f"{name:8s} M={M} N={N} K={K} " + " ".join(f"{k}={v if isinstance(v, str) else round(v, 1)}"
                                                      for k, v in out.items()) + f"  {tf:.0f} TF/s", flush=True)
