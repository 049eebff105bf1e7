#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): output tokens/sec of `lmstudio.chat_model`-style greedy
generation on a random-init Llama-3-8B Q4_K_M GGUF, one engine replica per GPU.

    python bench.py --gpus N --steps K --warmup W [--concurrency B] [--prompt-len P]

One step = one continuous-batching decode step over B in-flight requests per GPU
(hipGraph replay + per-step scheduling + the host<-device next-token copy: the real
serving loop, nothing skipped). N > 1 is launched by torch.distributed.run, one rank per
GPU; every rank is an independent replica (the reference's NATS queue-group scale-out,
README.md:478-484), so scaling is weak (fixed per-GPU work). Rank 0 prints ONE JSON line;
`value` is the whole-job aggregate (sum over ranks of tokens / max-over-ranks time).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "output tokens/sec + p50 NATS req-reply RTT, Llama-3-8B Q4_K chat_model"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--concurrency", type=int, default=512, help="in-flight chat requests per GPU")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--ftype", default="Q4_K_M")
    ap.add_argument("--model-dir", default=os.environ.get("NLS_BENCH_DIR", "/tmp/nls_bench"))
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-rtt", action="store_true")
    ap.add_argument("--single-stream", action="store_true", help="also time batch-1 decode (reported, not the headline)")
    ap.add_argument("--step-breakdown", action="store_true",
                    help="report host time vs time blocked on the previous step's tokens (diagnostic)")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from nats_llm_studio_amd import build as nbuild
    from nats_llm_studio_amd.gguf.reader import GGUFReader
    from nats_llm_studio_amd.gguf.synth import write_synthetic_gguf
    from nats_llm_studio_amd.models.llama import LlamaModel
    from nats_llm_studio_amd.engine.engine import Engine, GenRequest
    from nats_llm_studio_amd.engine.sampling import SamplingParams

    path = os.path.join(args.model_dir, f"{args.model}-{args.ftype}.gguf")
    t0 = time.time()
    if local == 0:
        nbuild.build_kernels()
        if not os.path.exists(path):
            os.makedirs(args.model_dir, exist_ok=True)
            write_synthetic_gguf(path, args.model, args.ftype, seed=0)
    if world > 1:
        dist.barrier()
    t_gen = time.time() - t0

    t0 = time.time()
    reader = GGUFReader(path)
    model = LlamaModel(reader, dev)
    torch.cuda.synchronize()
    t_load = time.time() - t0

    B = args.concurrency
    max_prefill = 2048
    # sequences prefilled early already decode while later ones prefill: budget those steps too
    prefill_steps = (B * args.prompt_len + max_prefill - 1) // max_prefill
    gen_tokens = args.warmup + args.steps + prefill_steps + 8
    need_tokens = args.prompt_len + gen_tokens
    eng = Engine(model, None, max_batch=B, max_prefill_tokens=max_prefill, use_graphs=not args.no_graphs,
                 ctx=max(need_tokens + 16, 512), num_blocks=B * ((need_tokens + 15) // 16 + 1))
    eng.capture_all()
    rng = np.random.default_rng(rank)
    vocab = model.cfg.vocab
    futs = [eng.submit(GenRequest(list(rng.integers(0, min(vocab, 100000), args.prompt_len)),
                                  SamplingParams(max_tokens=gen_tokens, ignore_eos=True)))
            for _ in range(B)]
    # prefill every request (not timed), then warm up the decode loop
    t0 = time.time()
    while any(s.n_prefilled < s.n_prompt for s in eng.running) or eng.waiting:
        eng.step()
    torch.cuda.synchronize()
    t_prefill = time.time() - t0
    for _ in range(args.warmup):
        eng.step()
    assert len(eng.running) == B, "all requests must still be decoding in the timed region"

    wait = [0.0]
    if args.step_breakdown:   # time the host spends blocked on step N's event (GPU-bound share)
        orig = eng._process

        def timed(infl):
            eng._ev[infl[1]].synchronize() if eng.dev.type == "cuda" else None
            t = time.perf_counter()
            orig(infl)
            wait[0] -= time.perf_counter() - t
        def timed_outer(infl):
            t = time.perf_counter()
            timed(infl)
            wait[0] += time.perf_counter() - t
        eng._process = timed_outer
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tokens = B * args.steps
    if args.step_breakdown:
        eng._process = orig
        eng._drain()
        # steady-state replay of the same decode graph, GPU-only (diagnostic: the replays rewrite
        # the last step's KV slots; nothing after this point is checked)
        g = eng.graphs.get((eng._bucket(B), False))
        if g is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            g.replay()
            e0.record()
            for _ in range(10):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            wait.append(e0.elapsed_time(e1) / 10)

    t_max = elapsed
    tok_sum = tokens
    if world > 1:
        tt = torch.tensor([elapsed, float(tokens)], dtype=torch.float64, device=dev)
        mx = tt.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        t_max = float(mx[0])
        tok_sum = float(tt[1])

    # drain
    while eng.running or eng.waiting:
        eng.step()
    for f in futs:
        f.result()

    extra = {}
    if args.step_breakdown:
        extra["step_breakdown_ms"] = {"gpu_wait": round(wait[0] / args.steps * 1e3, 3),
                                      "host_other": round((elapsed - wait[0]) / args.steps * 1e3, 3),
                                      "graph_replay_only": round(wait[1], 3) if len(wait) > 1 else None}
    if args.single_stream:
        r = eng.generate(list(rng.integers(0, 1000, args.prompt_len)), SamplingParams(max_tokens=64, ignore_eos=True))
        extra["single_stream_tok_s"] = round(r.tokens_per_second, 1)
        extra["single_stream_ttft_ms"] = round(r.time_to_first_token * 1e3, 2)

    rtt = None
    chat_rtt = None
    if not args.no_rtt and rank == 0:
        try:
            from nats_llm_studio_amd.service.bench_rtt import measure_rtt
            rtt = measure_rtt(n=500)
        except Exception as e:  # natscore missing -> report null, never fake
            extra["rtt_error"] = str(e)[:200]
        try:   # chat_model on the real 8B engine (after the timed region; engine idle)
            from nats_llm_studio_amd.service.bench_rtt import measure_engine_chat_rtt
            chat_rtt = measure_engine_chat_rtt(eng, reader.metadata, n=30)
        except Exception as e:
            extra["chat_rtt_error"] = str(e)[:300]

    if rank == 0:
        value = tok_sum / t_max
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "output tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp16",   # f16 activations + f16 MFMA on Q4_K_M weights, fp32 accumulate and residual
            "data": "synthetic prompts, random-init GGUF weights (Q4_K_M mix: Q4_K + Q6_K), no network",
            "config": {
                "model": f"{args.model} {args.ftype}",
                "global_batch": B * world,
                "seq_len": args.prompt_len,
                "parallelism": f"dp{world}",
                "concurrency_per_gpu": B,
                "hipgraph": not args.no_graphs,
            },
            "p50_rtt_ms": (chat_rtt or {}).get("p50_ms", None if rtt is None else rtt.get("p50_ms")),
            "rtt_chat_model_engine": chat_rtt,
            "rtt": rtt,
            "weights_gb": round(model.weight_bytes / 1e9, 3),
            "timings_s": {"gguf_write": round(t_gen, 1), "load": round(t_load, 1), "prefill_all": round(t_prefill, 3)},
            **extra,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
