#!/usr/bin/env python3
"""Sweep launch configs of the quantised GEMV/GEMM kernels on the real model shapes and
write the per-shape winners to nats_llm_studio_amd/ops/gemv_tuning.json.

Each config is timed as a hipGraph of REPS back-to-back launches (so host launch cost is
excluded), median of 5 replays. Usage: python tools/tune_gemv.py [--model llama-3-8b] [--out f.json]

--dense: tune the dense f16 GEMM (mode 4, weights' f16 copies) at the large-M buckets instead, next to
the current quantised winner of the same shape ("d:<rows>:<K>:<Mbucket>" entries).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np
import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.gguf import quants as Q
from nats_llm_studio_amd.gguf.constants import GGMLType
from nats_llm_studio_amd.gguf.synth import SPECS
from nats_llm_studio_amd.ops import tuning

REPS = 20


def shapes(spec, base=GGMLType.Q4_K, more=GGMLType.Q6_K):
    d, hd = spec.d_model, spec.head_dim
    nq, nkv = spec.n_head * hd, spec.n_kv_head * hd
    out = [
        ("qkv", [(base, nq), (base, nkv), (base, nkv)], d, "f32"),
        ("qkv6", [(base, nq), (base, nkv), (more, nkv)], d, "f32"),
        ("o", [(base, d)], nq, "add"),
        ("gateup", [(base, 2 * spec.d_ff)], d, "swiglu"),
        ("down", [(base, d)], spec.d_ff, "add"),
        ("down6", [(more, d)], spec.d_ff, "add"),
        ("lm_head", [(more, spec.vocab)], d, "argmax"),
    ]
    return out


def configs(K, M=1, quant=True):
    nb = K // 256
    if M > 64:   # large-M GEMM: path B (128-row activation blocks) or the LDS-dequant GEMM (mode 2)
        c = [(1, 4, 2, 1)]
        for ks in (1, 2, 3, 4, 6, 8):
            if ks <= max(1, nb // 2):
                c += [(1, 8, 1, ks), (1, 8, 2, ks)]
                if quant:
                    c += [(2, 8, 4, ks), (2, 8, 2, ks), (3, 4, 16, ks), (3, 4, 8, ks), (3, 4, 6, ks), (3, 4, 4, ks)]
                    if M >= 128:   # mode 9 (qgemm9.hip): 256 activation rows x 128 / 256 weight rows (8 waves),
                        # 128 weight rows on 4 waves (one per SIMD, 512 registers)
                        c += [(9, 8, 1, ks), (9, 8, 2, ks), (9, 4, 2, ks)]
        return c
    c = [(0, 8, 1, 1), (0, 4, 1, 1), (0, 8, 2, 1), (0, 4, 2, 1)]
    for waves in (4, 8):
        for rt in (1, 2):
            for ks in (1, 2, 4, 8, 16):
                if ks <= max(1, nb // 2):
                    c.append((1, waves, rt, ks))
    return c


def dense_configs(K):
    nkt = K // 64
    return ([(mode, wv, wm, ks) for mode in (5, 4) for wv in (8, 16) for wm in (4, 2) for ks in range(1, 9)
             if ks == 1 or nkt // ks >= 4]
            + [(6, 8, 2, ks) for ks in range(1, 9) if ks == 1 or nkt // ks >= 4])


def time_cfg(copies, x, y, M, epi, keys, cfg):
    """copies: weight-copy segment lists cycled through by the REPS launches, so small matrices are
    streamed from HBM as in a real decode step (one copy would sit in L2 / the 256 MB MALL)."""
    mode, waves, rt, ks = cfg
    kw = dict(mode=mode, waves=waves, rt=rt, ks=ks)
    e = "f32" if epi == "argmax" else epi
    am = keys if epi == "argmax" else None
    try:
        ops.qgemv(copies[0], x, y, M, epi=e, argmax=am, **kw)      # warm (allocates workspace)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(REPS):
                ops.qgemv(copies[i % len(copies)], x, y, M, epi=e, argmax=am, **kw)
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
        del g
        return sorted(ts)[2]
    except RuntimeError as ex:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--ms", default="1,2,4,8,16,32,48,64")
    ap.add_argument("--out", default=tuning._PATH)
    ap.add_argument("--log", default="gpurun_out/tune_gemv.log")
    ap.add_argument("--only", default="", help="comma list of shape names (qkv,qkv6,o,gateup,down,down6,lm_head)")
    ap.add_argument("--dense", action="store_true", help="tune mode 4 (dense f16) at M > 64")
    ap.add_argument("--modes", default="", help="comma list: time only these kernel modes (e.g. 9,11)")
    ap.add_argument("--base", default="q4_k", choices=("q4_k", "q5_k"),
                    help="base tile type of the shapes (Q4_K_M models: q4_k; Q5_K_M, e.g. Mixtral: q5_k)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    spec = SPECS[args.model]
    rng = np.random.default_rng(0)
    table = {}
    if os.path.exists(args.out):
        table = json.load(open(args.out))
    os.makedirs(os.path.dirname(args.log) or ".", exist_ok=True)
    log = open(args.log, "a")
    Ms = [int(m) for m in args.ms.split(",")]
    base = GGMLType.Q5_K if args.base == "q5_k" else GGMLType.Q4_K
    for name, segdef, K, epi in shapes(spec, base=base):
        if args.only and name not in args.only.split(","):
            continue
        segs, col = [], 0
        nbytes = 0
        for t, rows in segdef:
            raw = Q.random_blocks(t, rows * K, 0.02, rng)
            w = ops.QWeight(raw, t, rows, K, dev)
            nbytes += w.nbytes
            segs.append(ops.Seg(w, col))
            col += rows
        # enough copies that the timed launches stream > 1 GB (beyond the MALL), <= REPS copies
        ncopy = min(REPS, max(1, -(-(1 << 30) // nbytes)))
        copies = [segs] + [[ops.Seg(ops.QWeight.__new__(ops.QWeight), s.ycol) for s in segs] for _ in range(ncopy - 1)]
        for cp in copies[1:]:
            for s_new, s_old in zip(cp, segs):
                w = s_new.w
                w.__dict__.update(s_old.w.__dict__)
                w.data = s_old.w.data.clone()
        if args.dense:
            for cp in copies:       # Q|K|V copies as one buffer, as the model loads them (one merged segment)
                for s_ in cp:
                    s_.w.d16 = None
                ops.QWeight.expand_dense_group([s_.w for s_ in cp])
        ncol = col // 2 if epi == "swiglu" else col
        mmax = max(64, max(Ms))
        x = torch.randn(mmax, K, device=dev).to(ops.ACT_DTYPE)
        y = torch.zeros(mmax, ncol, dtype=ops.ACT_DTYPE if epi == "swiglu" else torch.float32, device=dev)
        keys = torch.zeros(mmax, dtype=torch.int64, device=dev)
        for M in Ms:
            res = []
            if args.dense:
                qcfg = tuning.select(segs, M)
                qus = time_cfg(copies, x, y, M, epi, keys, tuple(qcfg))
                modes = {int(m) for m in args.modes.split(",")} if args.modes else None
                cands = dense_configs(K)
                cur = tuning.select_dense(segs, M)      # the current entry (e.g. a mode-10 winner of dense_tune.py)
                if cur is not None and tuple(cur) not in cands:
                    cands.append(tuple(cur))
                for cfg in cands:
                    if modes is not None and cfg[0] not in modes and tuple(cfg) != tuple(cur or ()):
                        continue
                    us = time_cfg(copies, x, y, M, epi, keys, cfg)
                    if us is not None:
                        res.append((us, cfg))
                res.sort()
                best_us, best = res[0]
                # [-1]: the quantised GEMM measured faster for this shape and batch bucket
                table[tuning.dense_key(segs, M)] = list(best) if qus is None or best_us < qus else [-1]
                tf = 2.0 * M * col * K
                if qus is None:             # the quantised config failed to launch: the dense one wins by default
                    qus = float("inf")
                line = (f"{name:8s} M={M:4d} quant {tuple(qcfg)} {qus:8.2f}us {tf / qus / 1e6:7.1f} TF | dense best={best} "
                        f"{best_us:8.2f}us {tf / best_us / 1e6:7.1f} TF x{qus / best_us:4.2f} | "
                        + " ".join(f"{c}:{u:.1f}" for u, c in res[:4]))
                print(line, flush=True)
                log.write(line + "\n")
                log.flush()
                continue
            modes = {int(m) for m in args.modes.split(",")} if args.modes else None
            for cfg in configs(K, M, all(int(t) in (8, 12, 13, 14) for t, _ in segdef)):
                if modes is not None and cfg[0] not in modes:
                    continue
                us = time_cfg(copies, x, y, M, epi, keys, cfg)
                if us is not None:
                    res.append((us, cfg))
            res.sort()
            best_us, best = res[0]
            k = tuning.key(segs, M)
            table[k] = list(best)
            tf = 2.0 * M * col * K / best_us / 1e6
            line = (f"{name:8s} M={M:3d} best={best} {best_us:8.2f}us {nbytes / best_us / 1e3:7.1f} GB/s "
                    f"{tf:7.1f} TFLOP/s | "
                    + " ".join(f"{c}:{u:.1f}" for u, c in res[:4]))
            print(line, flush=True)
            log.write(line + "\n")
            log.flush()
        del segs, copies
        torch.cuda.empty_cache()
    with open(args.out, "w") as f:
        json.dump(table, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
