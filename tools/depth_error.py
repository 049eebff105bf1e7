#!/usr/bin/env python3
"""Where does the engine's logit error against the fp32 oracle come from? Prefill logits of the first n
layers (n = 1, 2, 4, ...) of a model against models/reference.py truncated the same way, plain fp32 and
with the engine's storage roundings; also the two oracles against each other (how much a rounding-sized
perturbation grows through n random-init layers).

    python tools/depth_error.py [--model llama-3-8b] [--S 512] [--depths 1,2,4,8,16,32] [--dense 0|1]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np
import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.gguf.reader import GGUFReader
from nats_llm_studio_amd.gguf.synth import write_synthetic_gguf
from nats_llm_studio_amd.models.llama import LlamaModel
from nats_llm_studio_amd.models.reference import ReferenceModel


def prefill_logits(model, ids):
    S = len(ids)
    nb = (S + 15) // 16
    b = model.step_buffers(S, S, nb)
    kc, vc = model.kv_cache(nb, 16)
    b.ids[:S] = torch.tensor(ids, dtype=torch.int32)
    b.pos[:S] = torch.arange(S)
    b.slot[:S] = torch.arange(S)
    b.tok_seq[:S] = 0
    b.ctx_len[:S] = torch.arange(S) + 1
    b.block_tables[0, :nb] = torch.arange(nb)
    qb = torch.from_numpy(ops.prefill_blocks(np.zeros(S, np.int32), np.arange(S, dtype=np.int32), S)).to(model.device)
    model.forward(b, kc, vc, S, 16, 1, qblocks=qb, nqb=len(qb))
    out = b.logits[:S].float().cpu()
    del b, kc, vc
    torch.cuda.empty_cache()
    return out


def rel(a, b):
    return (a - b).norm().item() / b.norm().item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--ftype", default="Q4_K_M")
    ap.add_argument("--S", type=int, default=512)
    ap.add_argument("--depths", default="1,2,4,8,16,32")
    ap.add_argument("--dense", type=int, default=0)
    a = ap.parse_args()
    d = os.environ.get("NLS_BENCH_DIR", "/tmp/nls_bench")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"{a.model}-{a.ftype}.gguf")
    if not os.path.exists(path):
        write_synthetic_gguf(path, a.model, a.ftype, seed=0)
    dev = torch.device("cuda:0")
    m = LlamaModel(GGUFReader(path), dev)
    if a.dense:
        m.expand_dense(None)
    else:
        ops.DENSE_MIN_M = 1 << 30
    full = list(m.layers)
    rd = GGUFReader(path)
    ids = [int(t) for t in np.random.default_rng(11).integers(0, min(128000, m.cfg.vocab), a.S)]
    for n in [int(v) for v in a.depths.split(",")]:
        m.layers = full[:n]
        got = prefill_logits(m, ids)
        refs = []
        for rnd in (False, True):
            r = ReferenceModel(rd, device=dev, cache=False, workers=16, storage_rounding=rnd)
            r.cfg.n_layer = n
            refs.append(r.logits(ids).float().cpu())
            torch.cuda.empty_cache()
        f, s = refs
        print(f"layers {n:3d}: engine vs fp32 {rel(got, f):.3e} vs storage-rounded {rel(got, s):.3e} | "
              f"storage-rounded vs fp32 {rel(s, f):.3e} | top-1 {(got.argmax(1) == f.argmax(1)).float().mean():.3f} "
              f"| |logits| {f.norm() / f.numel() ** 0.5:.3f}", flush=True)


if __name__ == "__main__":
    main()
