#!/usr/bin/env python3
"""Time-to-first-token of long single prompts on the real engine (chunked MFMA prefill: dense GEMMs on the
f16 copies + attn_prefill over the paged KV), and -- with --breakdown -- a per-kernel split of one prefill
from a rocprofv3 kernel trace taken around it.

    python tools/prefill_probe.py --lens 8192 32768 [--model llama-3.1-8b] [--kv bf16|fp8] [--reps 2]
    rocprofv3 --kernel-trace --stats -d gpurun_out/pf -o run --output-format csv -- python3 tools/prefill_probe.py ...
    python tools/prefill_probe.py --analyze gpurun_out/pf/.../run_kernel_trace.csv --lens 32768
"""
import argparse
import csv
import json
import os
import re
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def attn_flops(P: int, chunk: int, L: int, Hq: int, D: int) -> float:
    """Causal attention FLOPs of a P-token prompt prefilled in `chunk`-token pieces (QK^T + PV, 4 * D per
    query-key pair, keys up to and including the query's position)."""
    pairs = P * (P + 1) / 2
    return 4.0 * D * Hq * L * pairs


def run(a):
    import numpy as np
    import torch
    from nats_llm_studio_amd.engine.engine import Engine, GenRequest
    from nats_llm_studio_amd.engine.sampling import SamplingParams
    from nats_llm_studio_amd.gguf.reader import GGUFReader
    from nats_llm_studio_amd.gguf.synth import write_synthetic_gguf
    from nats_llm_studio_amd.models.llama import LlamaModel
    os.environ["NLS_KV_DTYPE"] = a.kv
    path = os.path.join(a.dir, f"{a.model}-Q4_K_M.gguf")
    if not os.path.exists(path):
        os.makedirs(a.dir, exist_ok=True)
        write_synthetic_gguf(path, a.model, "Q4_K_M", seed=0)
    dev = torch.device("cuda:0")
    m = LlamaModel(GGUFReader(path), dev)
    P = max(a.lens)
    eng = Engine(m, None, max_batch=4, max_prefill_tokens=a.chunk, ctx=P + 64, num_blocks=(P + 64) // 16 * 2 + 64)
    rng = np.random.default_rng(0)
    out = []
    for n in a.lens:
        for rep in range(a.reps):
            ids = [int(t) for t in rng.integers(0, 100000, n)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = eng.generate(ids, SamplingParams(max_tokens=1, ignore_eos=True))
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            cfg = m.cfg
            fl = attn_flops(n, a.chunk, cfg.n_layer, cfg.n_head, cfg.head_dim)
            out.append(dict(prompt=n, rep=rep, ttft_s=round(dt, 4), attn_tflop=round(fl / 1e12, 2), kv=a.kv,
                            chunk=a.chunk, tokens=len(r.token_ids)))
            print(json.dumps(out[-1]), flush=True)
    return out


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name).strip()[:80]


def analyze(path, P, model):
    from nats_llm_studio_amd.gguf.synth import SPECS
    spec = SPECS[model]
    rows = list(csv.DictReader(open(path)))
    agg, cnt = defaultdict(float), defaultdict(int)
    for r in rows:
        k = short(r["Kernel_Name"])
        agg[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
        cnt[k] += 1
    tot = sum(agg.values())
    print(f"kernel time total {tot:.3f} s over {sum(cnt.values())} launches")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:25]:
        print(f"{v:9.4f} s {100 * v / tot:5.1f} %  x{cnt[k]:6d}  {k}")
    at = sum(v for k, v in agg.items() if "attn_prefill" in k)
    if at > 0:
        fl = attn_flops(P, 2048, spec.n_layer, spec.n_head, spec.head_dim)
        n_prefills = max(1, round(cnt[[k for k in agg if "attn_prefill" in k][0]] / (spec.n_layer * ((P + 2047) // 2048))))
        print(f"attn_prefill: {at:.4f} s for {n_prefills} prefill(s) of {P} -> {n_prefills * fl / at / 1e12:.0f} TFLOP/s")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", type=int, nargs="+", default=[8192, 32768])
    ap.add_argument("--model", default="llama-3.1-8b")
    ap.add_argument("--kv", default="bf16")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--chunk", type=int, default=2048)
    ap.add_argument("--dir", default=os.environ.get("NLS_BENCH_DIR", "/tmp/nls_bench"))
    ap.add_argument("--analyze", default=None)
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze, max(a.lens), a.model)
    else:
        run(a)
