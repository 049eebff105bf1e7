#!/usr/bin/env python3
"""Debug probe: decode attention over an fp8 (e4m3) cache with one key (output == that V row)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from nats_llm_studio_amd import ops

dev = torch.device("cuda:0")
Hq, Hkv, D, bs = 4, 1, 128, 16
vals = torch.tensor([0.5, 1.0, 1.5, 2.0, -3.0, 0.25, 4.0, -0.125] * (D // 8))
for kvt in (torch.bfloat16, torch.float8_e4m3fn):
    kc = torch.zeros(bs, Hkv, D).to(kvt)
    vc = torch.zeros(bs, Hkv, D)
    vc[0, 0] = vals
    vc = vc.to(kvt)
    q = torch.randn(1, Hq * D).to(torch.bfloat16)
    bt = torch.zeros(1, 4, dtype=torch.int32)
    out = torch.zeros(1, Hq * D, dtype=ops.ACT_DTYPE, device=dev)
    ops.attention(q.to(dev), kc.to(dev), vc.to(dev), bt.to(dev), torch.zeros(1, dtype=torch.int32, device=dev),
                  torch.ones(1, dtype=torch.int32, device=dev), out, 1, Hq, Hkv, D, bs, D ** -0.5)
    torch.cuda.synchronize()
    print(kvt, "raw bytes", vc.view(torch.uint8)[0, 0, :8].tolist(), "out", out[0, :8].float().cpu().tolist(),
          "want", vc[0, 0, :8].float().tolist())
