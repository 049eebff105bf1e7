#!/usr/bin/env python3
"""Mode 8 (csrc/kernels/hgemm8.hip) against hipBLASLt and the current production launch, in ONE process,
at the Llama-3-8B projection shapes: every launch is captured in a hipGraph over rotating weight copies
(>= 1 GiB in flight, so weights stream from HBM as in decode) and timed as the median of rounds.

  * lib:   torch.mm (hipBLASLt) on the same f16 copy, GEMM only (no epilogue pass)
  * prod:  ops.gemv_config's launch with the shape's fused epilogue (what the engine runs today)
  * m8:    every mode-8 (rt, ks) candidate with the same fused epilogue; the best is reported and, with
           --emit, written as "d8:" tuning entries (JSON on stdout, tools/README.md)
  * m9:    every mode-9 (rt, ks) candidate (qgemm9.hip: the quantised tile-blocks, no f16 copy)

    python tools/hg8_ab.py --M 256,512,1024,2048 [--shapes qkv,o,gateup,down,lm_head] [--emit]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np
import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.gguf import quants as Q
from nats_llm_studio_amd.gguf.synth import SPECS

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


def graph_of(fn):
    fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(REPS):
            fn(i)
    return g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="256,512,1024,2048")
    ap.add_argument("--shapes", default="qkv,o,gateup,down,lm_head")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--cands", default="8:1,8:2,8:4,7:1,7:2,4:1,4:2,4:4,8:8,4:8")
    ap.add_argument("--cands9", default="8:2:1,8:2:2,8:2:4,8:2:8,8:1:1,8:1:2,8:1:4,4:2:1,4:2:2,4:2:4")
    ap.add_argument("--cands10", default="1,2,3,4,6,8", help="mode-10 split-K candidates")
    ap.add_argument("--types", default="", help="override the weight format of every shape (e.g. 14 = Q6_K)")
    ap.add_argument("--emit", action="store_true")
    a = ap.parse_args()
    spec = SPECS[a.model]
    d, hd = spec.d_model, spec.head_dim
    nq, nkv = spec.n_head * hd, spec.n_kv_head * hd
    defs = {"qkv": ([(12, nq), (12, nkv), (12, nkv)], d, "f32"), "o": ([(12, d)], nq, "add"),
            "gateup": ([(12, 2 * spec.d_ff)], d, "swiglu"), "down": ([(12, d)], spec.d_ff, "add"),
            "lm_head": ([(14, spec.vocab)], d, "argmax")}
    cands = [tuple(int(v) for v in c.split(":")) for c in a.cands.split(",") if c]
    cands9 = [tuple(int(v) for v in c.split(":")) for c in a.cands9.split(",") if c]
    cands10 = [int(c) for c in a.cands10.split(",") if c]
    if a.types:
        defs = {k: ([(int(a.types), r) for _, r in sd], K, e) for k, (sd, K, e) in defs.items()}
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    emit = {}
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
                w.d16 = s.w.d16.clone()
                w.data = s.w.data.clone()
                cp.append(ops.Seg(w, s.ycol))
            copies.append(cp)
        wcat = [torch.cat([s.w.d16 for s in cp], 0) for cp in copies]
        for M in [int(m) for m in a.M.split(",")]:
            flop = 2.0 * M * col * K
            x = (torch.randn(max(M, 64), K, device=dev) * 0.5).to(ops.ACT_DTYPE)
            ncol = col // 2 if epi == "swiglu" else col
            y = torch.zeros(max(M, 64), ncol, dtype=ops.ACT_DTYPE if epi == "swiglu" else torch.float32, device=dev)
            keys = torch.zeros(max(M, 64), dtype=torch.int64, device=dev)
            lib_out = torch.empty(max(M, 64), col, dtype=torch.float16, device=dev)
            ref = None

            def lib(i):
                torch.mm(x[:M], wcat[i % ncopy].t(), out=lib_out[:M])
            t_lib = timed(graph_of(lib), a.rounds)

            def launch(cfg):
                mode, waves, rt, ks = cfg
                if epi == "add":
                    nw = torch.ones(ncol, device=dev)
                    hn = torch.zeros(max(M, 64), ncol, dtype=ops.ACT_DTYPE, device=dev)

                    def fn(i):
                        ops.qgemv_add_rmsnorm(copies[i % ncopy][0], x, y, nw, hn, M, 1.0, 1e-5, cfg=cfg)
                elif epi == "argmax":
                    def fn(i):
                        ops.argmax_reset(keys)
                        ops.qgemv(copies[i % ncopy], x, y, M, epi="argmax", argmax=keys, mode=mode, waves=waves,
                                  rt=rt, ks=ks)
                else:
                    def fn(i):
                        ops.qgemv(copies[i % ncopy], x, y, M, epi=epi, mode=mode, waves=waves, rt=rt, ks=ks)
                return fn
            prod = ops.gemv_config(segs, M)
            try:
                t_prod = timed(graph_of(launch(prod)), a.rounds)
            except Exception as e:
                t_prod = float("nan")
                print(f"  prod {prod} failed: {e}")
            best = None
            for rt, ks in cands:
                if epi == "argmax" and ks > 1:
                    continue
                cfg = (8, 8, rt, ks)
                try:
                    t = timed(graph_of(launch(cfg)), a.rounds)
                except Exception as e:
                    print(f"  m8 {cfg} failed: {e}")
                    continue
                if best is None or t < best[0]:
                    best = (t, cfg)
            best9 = None
            for wv, rt, ks in cands9:
                if epi == "argmax" and ks > 1:
                    continue
                cfg = (9, wv, rt, ks)
                try:
                    t = timed(graph_of(launch(cfg)), a.rounds)
                except Exception as e:
                    print(f"  m9 {cfg} failed: {e}")
                    continue
                if best9 is None or t < best9[0]:
                    best9 = (t, cfg)
            best10 = None
            for ks in cands10:
                if epi == "argmax" and ks > 1:
                    continue
                cfg = (10, 8, 1, ks)
                try:
                    t = timed(graph_of(launch(cfg)), a.rounds)
                except Exception as e:
                    print(f"  m10 {cfg} failed: {e}")
                    continue
                if best10 is None or t < best10[0]:
                    best10 = (t, cfg)
            # correctness of the winner (plain f32 output vs the library's product)
            t8, cfg8 = best
            yy = torch.zeros(max(M, 64), col, device=dev)
            ops.qgemv(segs, x, yy, M, mode=8, waves=8, rt=cfg8[2], ks=cfg8[3])
            torch.mm(x[:M], wcat[0].t(), out=lib_out[:M])
            rel = float((yy[:M] - lib_out[:M].float()).abs().max() / (lib_out[:M].float().abs().max() + 1e-6))
            t10, cfg10 = best10 if best10 is not None else (float("nan"), None)
            t9, cfg9, rel9 = float("nan"), None, float("nan")
            if best9 is not None:
                t9, cfg9 = best9
                yy.zero_()
                ops.qgemv(segs, x, yy, M, mode=9, waves=cfg9[1], rt=cfg9[2], ks=cfg9[3])
                rel9 = float((yy[:M] - lib_out[:M].float()).abs().max() / (lib_out[:M].float().abs().max() + 1e-6))
            print(f"{name:8s} M={M:5d} lib {t_lib:8.2f}us {flop / t_lib / 1e6:7.1f}TF | prod{prod} {t_prod:8.2f}us | "
                  f"m8{cfg8} {t8:8.2f}us {flop / t8 / 1e6:7.1f}TF | m8/lib {t8 / t_lib:5.2f} m8/prod {t8 / t_prod:5.2f} "
                  f"| maxrel {rel:.1e} | m9{cfg9} {t9:8.2f}us {flop / t9 / 1e6:7.1f}TF m9/lib {t9 / t_lib:5.2f} "
                  f"maxrel {rel9:.1e} | m10{cfg10} {t10:8.2f}us {flop / t10 / 1e6:7.1f}TF m10/lib {t10 / t_lib:5.2f} "
                  f"m10/prod {t10 / t_prod:5.2f}", flush=True)
            emit[f"{name}:{M}"] = dict(cfg=list(cfg8), us=round(t8, 2), lib_us=round(t_lib, 2), prod=list(prod),
                                       prod_us=round(t_prod, 2), cfg9=list(cfg9) if cfg9 else None,
                                       us9=round(t9, 2), cfg10=list(cfg10) if cfg10 else None, us10=round(t10, 2))
    if a.emit:
        print(json.dumps(emit))


if __name__ == "__main__":
    main()
