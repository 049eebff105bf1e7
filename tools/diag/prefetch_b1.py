"""Batch-1 decode experiment: does a projection's GEMV run faster when its weights were just streamed into the
memory-side Infinity Cache (MALL) / L2 by a prefetch launch? Per Llama-3-8B shape at M=1 (tuned config):
  cold  -- REPS back-to-back GEMVs over distinct weight copies (> 1 GB: every launch streams from HBM)
  pf    -- the prefetch launch alone over the same copies (its HBM rate)
  pf+g  -- prefetch(copy i) then GEMV(copy i), serially; warm = (pf+g) - pf is the GEMV on cached weights
All times per launch, median of 5 hipGraph replays."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np
import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.gguf import quants as Q
from nats_llm_studio_amd.gguf.synth import SPECS
from nats_llm_studio_amd.ops import _lib, tuning
from tune_gemv import REPS, shapes


def timed(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        t.record()
        t.synchronize()
        ts.append(s.elapsed_time(t) / REPS * 1e3)
    return sorted(ts)[2]


def main():
    dev = torch.device("cuda:0")
    spec = SPECS["llama-3-8b"]
    rng = np.random.default_rng(0)
    L = _lib.lib()
    blocks = [int(b) for b in os.environ.get("PF_BLOCKS", "64,256").split(",")]
    for name, segdef, K, epi in shapes(spec):
        if name in ("lm_head", "qkv6", "down6"):
            continue
        segs, col, nbytes = [], 0, 0
        for t, rows in segdef:
            w = ops.QWeight(Q.random_blocks(t, rows * K, 0.02, rng), t, rows, K, dev)
            nbytes += w.nbytes
            segs.append(ops.Seg(w, col))
            col += rows
        copies = [segs]
        for _ in range(REPS - 1):
            cp = []
            for s in segs:
                w = ops.QWeight.__new__(ops.QWeight)
                w.__dict__.update(s.w.__dict__)
                w.data = s.w.data.clone()
                cp.append(ops.Seg(w, s.ycol))
            copies.append(cp)
        ncol = col // 2 if epi == "swiglu" else col
        x = torch.randn(1, K, device=dev).to(ops.ACT_DTYPE)
        y = torch.zeros(1, ncol, dtype=ops.ACT_DTYPE if epi == "swiglu" else torch.float32, device=dev)
        cfg = tuple(tuning.select(segs, 1))
        kw = dict(mode=cfg[0], waves=cfg[1], rt=cfg[2], ks=cfg[3])
        e = "f32" if epi == "add" else epi
        st = lambda: torch.cuda.current_stream().cuda_stream

        def gemv_all():
            for i in range(REPS):
                ops.qgemv(copies[i], x, y, 1, epi=e, **kw)
        cold = timed(gemv_all)
        line = f"{name:7s} {nbytes / 1e6:6.1f} MB cfg {cfg}: cold {cold:6.2f} us ({nbytes / cold / 1e3:5.0f} GB/s)"
        for nb in blocks:
            def pf_all():
                for i in range(REPS):
                    for s in copies[i]:
                        L.nls_prefetch(s.w.data.data_ptr(), s.w.data.numel() * s.w.data.element_size(), nb, st())

            def both():
                for i in range(REPS):
                    for s in copies[i]:
                        L.nls_prefetch(s.w.data.data_ptr(), s.w.data.numel() * s.w.data.element_size(), nb, st())
                    ops.qgemv(copies[i], x, y, 1, epi=e, **kw)
            pf = timed(pf_all)
            pg = timed(both)
            line += (f" | pf{nb} {pf:6.2f} us ({nbytes / pf / 1e3:5.0f} GB/s) pf+g {pg:6.2f} warm {pg - pf:6.2f} us"
                     f" ({nbytes / max(pg - pf, 1e-3) / 1e3:5.0f} GB/s)")
        print(line, flush=True)
        del copies, segs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
