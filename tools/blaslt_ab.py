#!/usr/bin/env python3
"""A/B in ONE process: the production large-M launch (ops/gemv_tuning.json: dense f16 modes 4-6 or the
quantised GEMM, epilogue fused) against hipBLASLt (torch.mm on the same f16 weight copies) followed by
the epilogue as a separate pass -- i.e. the library-GEMM alternative for the plain dense projections.
Weights rotate over copies (>= 1 GiB in flight) so every launch streams them from HBM, as in decode.

    python tools/blaslt_ab.py --M 256,512,1024 [--shapes qkv,o,gateup,down,lm_head]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np
import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.gguf import quants as Q
from nats_llm_studio_amd.gguf.synth import SPECS
from nats_llm_studio_amd.ops import tuning

REPS = 10


def timed(g, rounds):
    ts = []
    for _ in range(rounds):
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        g.replay()
        s1.record()
        s1.synchronize()
        ts.append(s0.elapsed_time(s1) / REPS * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="256,512,1024")
    ap.add_argument("--shapes", default="qkv,o,gateup,down,lm_head")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--model", default="llama-3-8b", help="projection shapes of this synthetic spec")
    ap.add_argument("--lib-ks", type=int, default=1, help="add shapes: the 'gemm only' column runs K-split "
                    "library GEMMs into slabs + the fused reduce/add/RMSNorm pass")
    a = ap.parse_args()
    spec = SPECS[a.model]
    d, hd = spec.d_model, spec.head_dim
    nq, nkv = spec.n_head * hd, spec.n_kv_head * hd
    defs = {"qkv": ([(12, nq), (12, nkv), (12, nkv)], d, "f32"), "o": ([(12, d)], nq, "add"),
            "gateup": ([(12, 2 * spec.d_ff)], d, "swiglu"), "down": ([(12, d)], spec.d_ff, "add"),
            "lm_head": ([(14, spec.vocab)], d, "f32")}
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    for name in a.shapes.split(","):
        segdef, K, epi = defs[name]
        segs, col = [], 0
        for t, rows in segdef:
            w = ops.QWeight(Q.random_blocks(t, rows * K, 0.02, rng), t, rows, K, dev)
            w.expand_dense()
            segs.append(ops.Seg(w, col))
            col += rows
        nbytes = col * K * 2
        ncopy = min(REPS, max(1, -(-(1 << 30) // nbytes)))
        copies = [segs]
        for _ in range(ncopy - 1):
            cp = []
            for s in segs:
                w = ops.QWeight.__new__(ops.QWeight)
                w.__dict__.update(s.w.__dict__)
                w.data = s.w.data.clone()
                w.d16 = s.w.d16.clone()
                cp.append(ops.Seg(w, s.ycol))
            copies.append(cp)
        for cp in copies:      # before any launch or capture (ops.fuse_dense: d16 pointers never move later)
            ops.fuse_dense(cp)
        # one [col, K] f16 matrix per copy for the library GEMM (segments concatenated: same bytes)
        wcat = [torch.cat([s.w.d16 for s in cp], 0) for cp in copies]
        for M in [int(m) for m in a.M.split(",")]:
            cfg = ops.gemv_config(segs, M)
            x = (torch.randn(max(M, 64), K, device=dev) * 0.5).to(ops.ACT_DTYPE)
            ncol = col // 2 if epi == "swiglu" else col
            y = torch.zeros(max(M, 64), ncol, dtype=ops.ACT_DTYPE if epi == "swiglu" else torch.float32,
                            device=dev)
            kw = dict(mode=cfg[0], waves=cfg[1], rt=cfg[2], ks=cfg[3])
            if epi == "add":       # o / down: residual add + next RMSNorm, as the decode step runs them
                nw = torch.rand(ncol, device=dev) + 0.5
                hn = torch.zeros(max(M, 64), ncol, dtype=ops.ACT_DTYPE, device=dev)

                def ours(i):
                    ops.qgemv_add_rmsnorm(copies[i % ncopy][0], x, y, nw, hn, M, 1.0, 1e-5, cfg=cfg)

                def lib(i):
                    ops.LIB_GEMM, tab = True, tuning.table()
                    key = tuning.lib_key(copies[i % ncopy], M)
                    old = tab.get(key)
                    tab[key] = (1,)
                    ops.qgemv_add_rmsnorm(copies[i % ncopy][0], x, y, nw, hn, M, 1.0, 1e-5)
                    tab.pop(key) if old is None else tab.__setitem__(key, old)
            else:
                def ours(i):
                    ops.qgemv(copies[i % ncopy], x, y, M, epi=epi, **kw)

                def lib(i):           # the production mode-7 path (HIP SwiGLU pass / f32 store)
                    ops.lib_gemm(copies[i % ncopy], x, y, M, 1.0, epi)
            ours(0)
            g1 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1):
                for i in range(REPS):
                    ours(i)

            def lib_gemm_only(i):
                if epi == "add" and a.lib_ks > 1:   # K split over slabs, then the fused reduce/norm pass
                    Wc, n = wcat[i % ncopy], ncol
                    ws = ops._workspace(dev, a.lib_ks * M * n)
                    kk = K // a.lib_ks
                    for j in range(a.lib_ks):
                        torch.mm(x[:M, j * kk:(j + 1) * kk], Wc[:, j * kk:(j + 1) * kk].t(), out_dtype=torch.float32,
                                 out=ws[j * M * n:(j + 1) * M * n].view(M, n))
                    ops._lib.check(ops._lib.lib().nls_splitk_add_rmsnorm(
                        ws.data_ptr(), a.lib_ks, M, 1.0, y.data_ptr(), y.stride(0), nw.data_ptr(), hn.data_ptr(),
                        hn.stride(0), n, 1e-5, ops._stream_ptr(x)), "splitk")
                    return
                torch.mm(x[:M], wcat[i % ncopy].t())

            outs = []
            for fn in (lambda: ours(0), lambda: lib(0)):
                y.zero_()
                fn()
                torch.cuda.synchronize()
                outs.append((hn if epi == "add" else y)[:M].float().clone())
            err = (outs[1] - outs[0]).abs().max().item() / (outs[0].abs().max().item() + 1e-9)
            graphs = [g1]
            for f in (lib, lib_gemm_only):
                f(0)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for i in range(REPS):
                        f(i)
                graphs.append(g)
            for g in graphs:
                g.replay()
            torch.cuda.synchronize()
            ts = [[] for _ in graphs]
            for _ in range(a.rounds):
                for gi, g in enumerate(graphs):
                    ts[gi].append(timed(g, 1))
            med = [sorted(t)[len(t) // 2] for t in ts]
            flops = 2.0 * M * col * K
            print(f"{name:8s} M={M:5d} ours{tuple(cfg)} {med[0]:8.2f}us {flops / med[0] / 1e6:6.1f}TF | "
                  f"hipBLASLt+epi {med[1]:8.2f}us | gemm only {med[2]:8.2f}us {flops / med[2] / 1e6:6.1f}TF | "
                  f"lib/ours {med[1] / med[0]:.2f} | maxrel {err:.1e}", flush=True)
            del graphs, g1
        del copies, segs, wcat
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
