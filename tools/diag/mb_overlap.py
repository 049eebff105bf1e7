"""Large-batch decode: would splitting the batch into two micro-batches whose layers run on two hipGraph
branches (one micro-batch's HBM-bound attention beside the other's compute-bound projections) beat one
full-batch chain? Llama-3-8B layer shapes with the f16 weight copies and the tuned large-M configs, bf16 K/V,
L distinct layers (weights and K/V stream from HBM), timed as hipGraph replays; per layer:
  full      -- one chain, B rows: Q|K|V, attention, o + add + norm, gate|up + SwiGLU, down + add + norm
  mb_serial -- two B/2-row chains back to back on one stream
  mb_branch -- the two B/2-row chains on two graph branches, B lagging A by one Q|K|V (an event edge per layer)
and, for the pairs that overlap in mb_branch, each op alone at B/2 rows vs two ops on two branches.
    python tools/diag/mb_overlap.py [--B 512] [--ctx 160] [--layers 4]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np
import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.gguf import quants as Q
from nats_llm_studio_amd.gguf.synth import SPECS
from nats_llm_studio_amd.models import llama


def graph_time(fn, reps=5):
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
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--ctx", type=int, default=160)
    ap.add_argument("--layers", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    spec = SPECS["llama-3-8b"]
    d, hd, dff = spec.d_model, spec.head_dim, spec.d_ff
    Hq, Hkv = spec.n_head, spec.n_kv_head
    nq, nkv = Hq * hd, Hkv * hd
    B, L, ctx, bs = a.B, a.layers, a.ctx, 16
    half = B // 2

    def qw(t, rows, K):
        w = ops.QWeight(Q.random_blocks(t, rows * K, 0.02, rng), t, rows, K, dev)
        w.expand_dense()
        return w
    base = dict(q=qw(12, nq, d), k=qw(12, nkv, d), v=qw(12, nkv, d), o=qw(12, d, nq), gu=qw(12, 2 * dff, d),
                dn=qw(12, d, dff))

    def clone(w):
        c = ops.QWeight.__new__(ops.QWeight)
        c.__dict__.update(w.__dict__)
        c.d16 = w.d16.clone()
        return c
    layers = []
    nbr = (ctx + bs - 1) // bs
    for l in range(L):
        ws = {k: (base[k] if l == 0 else clone(base[k])) for k in base}
        kc = (torch.randn(B * nbr * bs, Hkv, hd, device=dev) * 0.5).to(torch.bfloat16)
        layers.append(dict(qkv=[ops.Seg(ws["q"], 0), ops.Seg(ws["k"], nq), ops.Seg(ws["v"], nq + nkv)],
                           o=ops.Seg(ws["o"]), gu=[ops.Seg(ws["gu"])], dn=ops.Seg(ws["dn"]), kc=kc,
                           vc=torch.randn_like(kc)))
    bt_all = torch.arange(B * nbr, dtype=torch.int32, device=dev).view(B, nbr)

    def rows(n, off):
        ns = llama.LlamaModel.attn_splits(n, Hkv)
        return dict(n=n, ns=ns, x=(torch.randn(n, d, device=dev) * 0.5).to(ops.ACT_DTYPE),
                    xf=torch.randn(n, d, device=dev), qkv=torch.zeros(n, nq + 2 * nkv, device=dev),
                    q=torch.randn(n, nq, device=dev).to(torch.bfloat16),
                    att=torch.zeros(n, nq, dtype=ops.ACT_DTYPE, device=dev),
                    act=torch.zeros(n, dff, dtype=ops.ACT_DTYPE, device=dev),
                    h=torch.zeros(n, d, dtype=ops.ACT_DTYPE, device=dev), nw=torch.ones(d, device=dev),
                    bt=bt_all[off:off + n].contiguous(), ts=torch.arange(n, dtype=torch.int32, device=dev),
                    cl=torch.full((n,), ctx, dtype=torch.int32, device=dev),
                    ws=torch.zeros(n * Hq * ns * (hd + 2), device=dev),
                    cnt=torch.zeros(n * Hkv, dtype=torch.int32, device=dev))
    full, mA, mB = rows(B, 0), rows(half, 0), rows(half, half)

    def op(name, r, l):
        Ly = layers[l]
        n = r["n"]
        if name == "qkv":
            ops.qgemv(Ly["qkv"], r["x"], r["qkv"], n)
        elif name == "attn":
            ops.attention(r["q"], Ly["kc"], Ly["vc"], r["bt"], r["ts"], r["cl"], r["att"], n, Hq, Hkv, hd, bs,
                          hd ** -0.5, chunk=-llama._MIN_CHUNK, n_split=r["ns"], workspace=r["ws"],
                          counters=r["cnt"])
        elif name == "o":
            ops.qgemv_add_rmsnorm(Ly["o"], r["att"], r["xf"], r["nw"], r["h"], n, 1.0, 1e-5)
        elif name == "gu":
            ops.qgemv(Ly["gu"], r["h"], r["act"], n, epi="swiglu")
        elif name == "dn":
            ops.qgemv_add_rmsnorm(Ly["dn"], r["act"], r["xf"], r["nw"], r["x"], n, 1.0, 1e-5)
    OPS = ("qkv", "attn", "o", "gu", "dn")

    def chain(r):
        for l in range(L):
            for nm in OPS:
                op(nm, r, l)

    def branches(lag=True):
        main = torch.cuda.current_stream()
        sb = torch.cuda.Stream()
        sb.wait_stream(main)
        evs = []
        for l in range(L):
            for nm in OPS:
                op(nm, mA, l)
                if nm == "qkv" and lag:
                    e = torch.cuda.Event()
                    e.record(main)
                    evs.append(e)
        with torch.cuda.stream(sb):
            for l in range(L):
                if lag:
                    sb.wait_event(evs[l])
                for nm in OPS:
                    op(nm, mB, l)
        main.wait_stream(sb)

    t_full = graph_time(lambda: chain(full)) / L
    t_ser = graph_time(lambda: (chain(mA), chain(mB))) / L
    t_br = graph_time(branches) / L
    t_br0 = graph_time(lambda: branches(False)) / L
    print(f"B={B} ctx={ctx} layers={L}: per layer full {t_full:.1f} us | two {half}-row chains serial {t_ser:.1f} us | "
          f"on two branches, B lagging one Q|K|V {t_br:.1f} us | no lag {t_br0:.1f} us", flush=True)
    for nm in OPS:
        t1 = graph_time(lambda: [op(nm, full, l) for l in range(L)]) / L
        t2 = graph_time(lambda: [op(nm, mA, l) for l in range(L)]) / L
        print(f"  {nm:5s} alone: {B} rows {t1:7.1f} us, {half} rows {t2:7.1f} us", flush=True)

    def pair(n1, n2):
        main = torch.cuda.current_stream()
        sb = torch.cuda.Stream()
        sb.wait_stream(main)
        for l in range(L):
            op(n1, mA, l)
        with torch.cuda.stream(sb):
            for l in range(L):
                op(n2, mB, l)
        main.wait_stream(sb)
    for n1, n2 in (("attn", "qkv"), ("attn", "gu"), ("attn", "dn"), ("attn", "o"), ("gu", "dn")):
        t1 = graph_time(lambda: [op(n1, mA, l) for l in range(L)]) / L
        t2 = graph_time(lambda: [op(n2, mB, l) for l in range(L)]) / L
        tp = graph_time(lambda: pair(n1, n2)) / L
        print(f"  pair {n1}+{n2} ({half} rows each): alone {t1:.1f} + {t2:.1f} = {t1 + t2:.1f} us, on two branches "
              f"{tp:.1f} us ({(t1 + t2) / tp:.2f}x)", flush=True)


if __name__ == "__main__":
    main()
