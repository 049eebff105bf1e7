#!/usr/bin/env python3
"""Hand-written large-M GEMM launch configs for every dense projection shape of a model family, measured
against hipBLASLt (torch.mm on the same f16 copy, GEMM only -- a floor for the library path, which also
needs an epilogue pass). Every launch is captured in a hipGraph over rotating weight copies (>= 1 GiB, so
weights stream from HBM as in serving) and timed as the median of rounds.

Candidates: mode 10 (hgemm10.hip, 8-phase, 256 (rt 1) or 128 (rt 2) weight rows x 256 activation rows) x split-K, modes 4/5 (hgemm.hip, 128/256 weight rows,
128/256 activation rows, 8 or 16 waves) x split-K. With --emit the winners are printed as "d:<rows>:<K>:<Mbucket>" tuning
entries (ops/gemv_tuning.json) -- the table that replaced the library-GEMM ("L:") selections.

    python tools/dense_tune.py --model llama-3-70b --M 256,512,1024,2048 [--roles qkv,o,gateup,down,lm_head] --emit
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


def graph_of(fn):
    fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(REPS):
            fn(i)
    return g


def roles(spec):
    d, hd = spec.d_model, spec.head_dim
    nq, nkv = spec.n_head * hd, spec.n_kv_head * hd
    return {"qkv": ([(12, nq), (12, nkv), (12, nkv)], d, "f32"), "o": ([(12, d)], nq, "add"),
            "gateup": ([(12, 2 * spec.d_ff)], d, "swiglu"), "down": ([(12, d)], spec.d_ff, "add"),
            "lm_head": ([(14, spec.vocab)], d, "argmax")}


def candidates(M, K, epi):
    out = [(10, 8, rt, ks) for rt in (1, 2) for ks in (1, 2, 3, 4, 6, 8)]
    for mode in (4, 5):
        for waves in (8, 16):
            for wm in ((2, 4) if M >= 192 else (2,)):
                for ks in (1, 2, 4):
                    out.append((mode, waves, wm, ks))
    if epi == "argmax":
        out = [c for c in out if c[3] == 1]
    nkt = K // 64
    out = [c for c in out if nkt // c[3] >= 8]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--M", default="256,512,1024,2048")
    ap.add_argument("--roles", default="qkv,o,gateup,down,lm_head")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--emit", action="store_true")
    ap.add_argument("--modes", default="", help="comma list: time only these modes (e.g. 4,10)")
    a = ap.parse_args()
    spec = SPECS[a.model]
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    emit, rows_out = {}, []
    for name in a.roles.split(","):
        segdef, K, epi = roles(spec)[name]
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
            nw = torch.ones(ncol, device=dev)
            hn = torch.zeros(max(M, 64), ncol, dtype=ops.ACT_DTYPE, device=dev)

            def lib(i):
                torch.mm(x[:M], wcat[i % ncopy].t(), out=lib_out[:M])
            t_lib = timed(graph_of(lib), a.rounds)

            def launch(cfg):
                mode, waves, rt, ks = cfg
                if epi == "add":
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
            res = []
            for cfg in candidates(M, K, epi):
                if a.modes and cfg[0] not in {int(m) for m in a.modes.split(",")}:
                    continue
                try:
                    res.append((timed(graph_of(launch(cfg)), a.rounds), cfg))
                except Exception as e:
                    print(f"  {name} M={M} {cfg} failed: {e}", flush=True)
            res.sort()
            t_best, cfg_best = res[0]
            # correctness of the winner: plain f32 output against the library product
            yy = torch.zeros(max(M, 64), col, device=dev)
            ops.qgemv(segs, x, yy, M, mode=cfg_best[0], waves=cfg_best[1], rt=cfg_best[2], ks=cfg_best[3])
            torch.mm(x[:M], wcat[0].t(), out=lib_out[:M])
            rel = float((yy[:M] - lib_out[:M].float()).abs().max() / (lib_out[:M].float().abs().max() + 1e-6))
            line = dict(model=a.model, role=name, M=M, rows=col, K=K, lib_us=round(t_lib, 2),
                        lib_TF=round(flop / t_lib / 1e6, 1), hand_us=round(t_best, 2),
                        hand_TF=round(flop / t_best / 1e6, 1), cfg=list(cfg_best), hand_over_lib=round(t_best / t_lib, 3),
                        maxrel=float(f"{rel:.2e}"), runner_up=[[round(t, 2), list(c)] for t, c in res[1:4]],
                        all=[[round(t, 2), list(c)] for t, c in res])
            print(json.dumps(line), flush=True)
            rows_out.append(line)
            emit[tuning.dense_key(segs, M)] = list(cfg_best)
        del copies, wcat, segs
        torch.cuda.empty_cache()
    if a.emit:
        print("EMIT " + json.dumps(emit), flush=True)


if __name__ == "__main__":
    main()
