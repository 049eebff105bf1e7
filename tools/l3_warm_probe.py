"""Batch-1 GEMV time with the weights resident in the Infinity Cache (same weight every call) vs streamed
from HBM (cycling copies whose total exceeds 256 MiB), at the Llama-3-8B Q4_K_M shapes and their tuned
configs. The gap bounds what prefetching the next projection's weights into the L3 can buy at batch 1.
  python tools/l3_warm_probe.py [--sweep] [--shape qkv|o|gateup|down]  -> one JSON line per shape / config
"""
import copy
import json
import math

import numpy as np
import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.gguf import quants as Q
from nats_llm_studio_amd.ops import tuning

SHAPES = [("qkv", [12, 12, 12], 6144, 4096), ("o", [12], 4096, 4096), ("gateup", [12], 28672, 4096),
          ("down", [14], 4096, 14336)]


def segs_for(types, rows, K, rng):
    parts = [(types[0], rows - 2 * (rows // 6)), (types[1], rows // 6), (types[2], rows // 6)] if len(types) == 3 \
        else [(types[0], rows)]
    segs, col = [], 0
    for t, r in parts:
        segs.append(ops.Seg(ops.QWeight(Q.random_blocks(t, r * K, 0.02, rng), t, r, K, "cuda"), col))
        col += r
    return segs


def clone(segs):
    out = []
    for s in segs:
        w = copy.copy(s.w)
        w.data = s.w.data.clone()
        out.append(ops.Seg(w, s.ycol))
    return out


def timed(fn, reps=64, iters=5):
    g = torch.cuda.CUDAGraph()
    fn()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for i in range(reps):
            fn(i)
    best = math.inf
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / reps)
    return best


CFGS = [(1, 4, 2, 1), (1, 8, 1, 1), (1, 4, 1, 1), (1, 8, 2, 1), (1, 4, 2, 2), (1, 8, 1, 2), (0, 4, 1, 1),
        (0, 8, 1, 1), (0, 4, 2, 1), (0, 8, 2, 1), (0, 4, 1, 2), (1, 16, 1, 1)]


def main():
    import sys
    rng = np.random.default_rng(0)
    sweep = "--sweep" in sys.argv
    only = sys.argv[sys.argv.index("--shape") + 1] if "--shape" in sys.argv else None
    cfgs = [tuple(c) for c in json.loads(sys.argv[sys.argv.index("--cfgs") + 1])] if "--cfgs" in sys.argv else None
    for name, types, rows, K in SHAPES:
        if (sweep and name not in ("gateup", "down")) or (only and name != only):
            continue
        segs = segs_for(types, rows, K, rng)
        nbytes = sum(s.w.data.numel() * s.w.data.element_size() for s in segs)
        copies = [segs] + [clone(segs) for _ in range(max(1, math.ceil(640e6 / nbytes)) - 1)]
        x = torch.zeros(64, K, dtype=ops.ACT_DTYPE, device="cuda")
        x[0] = torch.randn(K, device="cuda").to(ops.ACT_DTYPE)
        y = torch.zeros(64, rows, device="cuda")
        for cfg in (cfgs or (CFGS if sweep else [tuning.select(segs, 1)])):
            mode, waves, rt, ks = cfg
            run = lambda c: ops.qgemv(c, x, y, 1, mode=mode, waves=waves, rt=rt, ks=ks)
            try:
                warm = timed(lambda i=0: run(segs))
                cold = timed(lambda i=0: run(copies[i % len(copies)]))
            except Exception as e:  # config not instantiated for this shape
                print(json.dumps({"shape": name, "cfg": list(cfg), "error": str(e)[:120]}), flush=True)
                continue
            print(json.dumps({"shape": name, "MB": round(nbytes / 1e6, 2), "cfg": list(cfg), "copies": len(copies),
                              "warm_us": round(warm, 2), "cold_us": round(cold, 2),
                              "warm_TBps": round(nbytes / warm / 1e6, 2), "cold_TBps": round(nbytes / cold / 1e6, 2)}),
                  flush=True)
        del copies, segs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
