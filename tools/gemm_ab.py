#!/usr/bin/env python3
"""A/B of kernel-library variants IN ONE PROCESS (interleaved rounds, cdna_hip_programming.md §5.4
rule 24): the production launch configs (ops/gemv_tuning.json) of the Llama-3-8B projections at batch M,
weights streamed from HBM (rotating copies), each variant timed as a hipGraph of REPS launches.

    python tools/gemm_ab.py --libs nats_llm_studio_amd/_kernels.so,nats_llm_studio_amd/_kernels_v1.so --M 512
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
from nats_llm_studio_amd.gguf.constants import GGMLType
from nats_llm_studio_amd.gguf.synth import SPECS
from nats_llm_studio_amd.ops import _lib, tuning

REPS = 10


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--M", type=int, default=512)
    ap.add_argument("--shapes", default="qkv,o,gateup,down,lm_head")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--dense", action="store_true", help="f16 weight copies: the large-M dense GEMM configs")
    a = ap.parse_args()
    libs = [(p, _lib.load(p)) for p in a.libs.split(",")]
    spec = SPECS["llama-3-8b"]
    d, hd = spec.d_model, spec.head_dim
    nq, nkv = spec.n_head * hd, spec.n_kv_head * hd
    defs = {"qkv": ([(12, nq), (12, nkv), (12, nkv)], d, "f32"), "o": ([(12, d)], nq, "add"),
            "gateup": ([(12, 2 * spec.d_ff)], d, "swiglu"), "down": ([(12, d)], spec.d_ff, "add"),
            "down6": ([(14, d)], spec.d_ff, "add"), "lm_head": ([(14, spec.vocab)], d, "f32")}
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    M = a.M
    for name in a.shapes.split(","):
        segdef, K, epi = defs[name]
        segs, col, nbytes = [], 0, 0
        for t, rows in segdef:
            w = ops.QWeight(Q.random_blocks(t, rows * K, 0.02, rng), t, rows, K, dev)
            if a.dense:
                w.expand_dense()
            nbytes += w.nbytes if not a.dense else w.dense_bytes
            segs.append(ops.Seg(w, col))
            col += rows
        ncopy = min(REPS, max(1, -(-(1 << 30) // nbytes)))
        copies = [segs]
        for _ in range(ncopy - 1):
            cp = []
            for s in segs:
                w = ops.QWeight.__new__(ops.QWeight)
                w.__dict__.update(s.w.__dict__)
                w.data = s.w.data.clone()
                if a.dense:
                    w.d16 = s.w.d16.clone()
                cp.append(ops.Seg(w, s.ycol))
            copies.append(cp)
        cfg = ops.gemv_config(segs, M)
        x = (torch.randn(max(M, 64), K, device=dev) * 0.5).to(ops.ACT_DTYPE)
        ncol = col // 2 if epi == "swiglu" else col
        y = torch.zeros(max(M, 64), ncol, dtype=ops.ACT_DTYPE if epi == "swiglu" else torch.float32, device=dev)
        graphs = []
        outs = []
        for path, L in libs:
            _lib._lib = L
            kw = dict(mode=cfg[0], waves=cfg[1], rt=cfg[2], ks=cfg[3])
            y.zero_()
            ops.qgemv(segs, x, y, M, epi=epi, **kw)
            torch.cuda.synchronize()
            outs.append(y[:M].float().clone())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(REPS):
                    ops.qgemv(copies[i % ncopy], x, y, M, epi=epi, **kw)
            g.replay()
            torch.cuda.synchronize()
            graphs.append(g)
        diffs = []
        for o in outs[1:]:
            err = (o - outs[0]).abs().max().item() / (outs[0].abs().max().item() + 1e-9)
            assert err < 1e-2, f"{name}: variant output differs ({err:.3g})"
            diffs.append("bit-equal" if torch.equal(o, outs[0]) else f"max rel diff {err:.2e}")
        ts = [[] for _ in libs]
        for _ in range(a.rounds):
            for li, g in enumerate(graphs):
                s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s0.record()
                g.replay()
                s1.record()
                s1.synchronize()
                ts[li].append(s0.elapsed_time(s1) / REPS * 1e3)
        flops = 2.0 * M * col * K
        line = f"{name:8s} M={M} cfg={cfg}"
        for (path, _), t in zip(libs, ts):
            med = sorted(t)[len(t) // 2]
            line += f" | {os.path.basename(path)} {med:8.2f}us {flops / med / 1e6:6.1f}TF"
        print(line + (" | " + ", ".join(diffs) if diffs else ""), flush=True)
        del graphs, copies, segs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
