"""Batch-1 decode: the fixed cost of one launch inside a captured hipGraph. Chains of N dependent launches on one
stream, captured once and replayed; per-link time of
  * a 1-element torch add (dispatch + completion of a trivial kernel),
  * M=1 Q4_K GEMVs x_{i+1} = f16(W_i x_i) with the tuned batch-1 config, W_i [R, 4096], R = 256 .. 14336
    (x_{i+1} takes the first 4096 outputs; rows beyond are written to a scratch tail),
and the least-squares line t = a + bytes / bw through the GEMV points: `a` is the per-launch cost a fused
(fewer-launch) decode layer could remove, `bw` the streaming rate.
Then the same chains with the weights held in the Infinity Cache (a few distinct weights cycled, > the 32 MiB of
L2, < its 256 MiB): how much of the per-link streaming time a read from the die-level cache instead of HBM saves
(the case for prefetching the next GEMV's weights into it while the current one runs)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np
import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.gguf import quants as Q
from nats_llm_studio_amd.gguf.constants import GGMLType


def per_link(fn, N, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / N)
    return float(np.median(ts))


def main(N=24, D=4096):
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    t = torch.zeros(1, device=dev)

    def tiny():
        for _ in range(N):
            t.add_(1.0)
    print(f"tiny add: {per_link(tiny, N):.2f} us per link", flush=True)

    pts = []
    for R in (256, 1024, 4096, 6144, 14336):
        ws = [ops.QWeight(Q.random_blocks(GGMLType.Q4_K, R * D, 0.02, rng), GGMLType.Q4_K, R, D, dev) for _ in range(N)]
        ys = [torch.zeros(16, max(R, D), dtype=ops.ACT_DTYPE, device=dev) for _ in range(N + 1)]
        ys[0][0, :D] = (torch.randn(D, device=dev) * 0.5).to(ops.ACT_DTYPE)
        cfg = ops.gemv_config([ops.Seg(ws[0])], 1)

        def chain():
            for i in range(N):
                ops.qgemv([ops.Seg(ws[i])], ys[i][:, :D], ys[i + 1], 1, epi="act")
        us = per_link(chain, N)
        nbytes = R * D * 144 // 256
        pts.append((nbytes, us))
        print(f"gemv R={R:6d} K={D} Q4_K cfg={cfg}: {us:.2f} us per link, {nbytes / us / 1e6:.2f} TB/s", flush=True)
        del ws, ys
        torch.cuda.empty_cache()
    b = np.array([p[0] for p in pts], dtype=np.float64)
    u = np.array([p[1] for p in pts])
    A = np.stack([np.ones_like(b), b], 1)
    (a, s), *_ = np.linalg.lstsq(A, u, rcond=None)
    print(f"fit: t = {a:.2f} us + bytes / {1 / s / 1e6:.2f} TB/s", flush=True)
    for R, nw in ((4096, 8), (6144, 6), (14336, 4)):
        ws = [ops.QWeight(Q.random_blocks(GGMLType.Q4_K, R * D, 0.02, rng), GGMLType.Q4_K, R, D, dev) for _ in range(nw)]
        ys = [torch.zeros(16, max(R, D), dtype=ops.ACT_DTYPE, device=dev) for _ in range(N + 1)]
        ys[0][0, :D] = (torch.randn(D, device=dev) * 0.5).to(ops.ACT_DTYPE)

        def chain():
            for i in range(N):
                ops.qgemv([ops.Seg(ws[i % nw])], ys[i][:, :D], ys[i + 1], 1, epi="act")
        us = per_link(chain, N)
        nbytes = R * D * 144 // 256
        print(f"gemv R={R:6d} resident ({nw} weights, {nw * nbytes / 2**20:.0f} MiB cycled): {us:.2f} us per link, "
              f"{nbytes / us / 1e6:.2f} TB/s, streaming part {us - a:.2f} us", flush=True)
        del ws, ys
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
