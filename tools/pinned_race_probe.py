#!/usr/bin/env python3
"""Does a non_blocking H2D copy from pinned host memory read the host buffer when the DMA EXECUTES (stream
order) rather than when it is enqueued? If so, rewriting the pinned buffer before the copy ran -- as a
prefill chunk's metadata did for the next chunk -- changes what the earlier chunk sees.
Prints {"seen": 1} (copy took the value at enqueue time) or {"seen": 2} (it read the later write)."""
import json

import torch

x = torch.randn(8192, 8192, device="cuda", dtype=torch.float16)
h = torch.zeros(1 << 16, dtype=torch.int32, pin_memory=True)
d = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
out = []
for size in (64, 1 << 16):
    h.fill_(1)
    for _ in range(20):                  # ~20 ms of queued GPU work ahead of the copy
        x = x @ x.t() * 1e-4
    d[:size].copy_(h[:size], non_blocking=True)
    h.fill_(2)                           # the host moves on and rewrites the staging buffer
    torch.cuda.synchronize()
    out.append(dict(elems=size, seen=int(d[0].item())))
print(json.dumps(out))
