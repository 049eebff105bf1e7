#!/usr/bin/env python3
"""KV capacity under on-demand allocation: N concurrent requests whose prompt + max_tokens far exceed the
KV pool (Llama-3-8B, default pool = half the free HBM after weights), decoded for a fixed wall time.
Reports, every few seconds and at the end: running / waiting sequences, KV blocks free, preemptions and
recomputed tokens, decode tok/s -- the concurrency the pool actually sustains.
    python tools/kv_pressure.py [--n 512] [--max-tokens 4096] [--seconds 60] [--reserve ondemand|full]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--max-tokens", type=int, default=4096)
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--reserve", default="ondemand", choices=("ondemand", "full"))
    ap.add_argument("--kv-fraction", type=float, default=0.5)
    a = ap.parse_args()
    os.environ["NLS_KV_RESERVE"] = a.reserve
    from nats_llm_studio_amd.engine.engine import Engine, GenRequest
    from nats_llm_studio_amd.engine.sampling import SamplingParams
    from nats_llm_studio_amd.gguf.reader import GGUFReader
    from nats_llm_studio_amd.gguf.synth import write_synthetic_gguf
    from nats_llm_studio_amd.models.llama import LlamaModel
    d = os.environ.get("NLS_BENCH_DIR", "/tmp/nls_bench")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"{a.model}-Q4_K_M.gguf")
    if not os.path.exists(path):
        write_synthetic_gguf(path, a.model, "Q4_K_M", seed=0)
    dev = torch.device("cuda:0")
    m = LlamaModel(GGUFReader(path), dev)
    ctx = min(m.cfg.ctx, a.prompt + a.max_tokens + 16)
    eng = Engine(m, None, max_batch=a.n, max_prefill_tokens=2048, ctx=ctx, kv_mem_fraction=a.kv_fraction)
    pool_tokens = eng.num_blocks * eng.bs
    need = a.n * (a.prompt + a.max_tokens)
    print(json.dumps(dict(pool_blocks=eng.num_blocks, pool_tokens=pool_tokens, demand_tokens=need,
                          demand_over_pool=round(need / pool_tokens, 2), reserve=a.reserve)), flush=True)
    rng = np.random.default_rng(0)
    futs = [eng.submit(GenRequest(list(rng.integers(0, 100000, a.prompt)),
                                  SamplingParams(max_tokens=a.max_tokens, ignore_eos=True))) for _ in range(a.n)]
    t0 = time.monotonic()
    last, c_last = t0, dict(eng.counters)
    peak = 0
    samples = []
    while time.monotonic() - t0 < a.seconds and not all(f.done() for f in futs):
        eng.step()
        peak = max(peak, len(eng.running))
        now = time.monotonic()
        if now - last >= 5.0:
            c = dict(eng.counters)
            rec = dict(t=round(now - t0, 1), running=len(eng.running), waiting=len(eng.waiting),
                       kv_free=eng.alloc.n_free, preemptions=c["preemptions"], recompute_tokens=c["recompute_tokens"],
                       decode_tok_s=round((c["decode_tokens"] - c_last["decode_tokens"]) / (now - last), 1))
            samples.append(rec)
            print(json.dumps(rec), flush=True)
            last, c_last = now, c
    torch.cuda.synchronize()
    el = time.monotonic() - t0
    c = eng.counters
    done = sum(f.done() for f in futs)
    ok = sum(1 for f in futs if f.done() and len(f.result().token_ids) == a.max_tokens)
    print(json.dumps(dict(summary=True, seconds=round(el, 1), peak_running=peak,
                          mean_running=round(float(np.mean([s["running"] for s in samples])), 1) if samples else peak,
                          finished=done, finished_full_length=ok, decode_tokens=c["decode_tokens"],
                          decode_tok_s=round(c["decode_tokens"] / el, 1), preemptions=c["preemptions"],
                          recompute_tokens=c["recompute_tokens"], prefill_tokens=c["prefill_tokens"],
                          # share of all forward tokens spent re-prefilling preempted sequences
                          recompute_waste=round(c["recompute_tokens"] / max(1, c["decode_tokens"] + c["prefill_tokens"]), 4),
                          pool_tokens=pool_tokens)), flush=True)
    eng.shutdown()


if __name__ == "__main__":
    main()
