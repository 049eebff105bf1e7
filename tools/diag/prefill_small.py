"""A short single-prompt prefill (the engine chat_model RTT case: ~21 prompt tokens, max_tokens 1) on the 8B: wall time of
eng.generate, and for the model forward inside it the HOST time of issuing its launches vs the GPU time between
events recorded around it. host >= gpu means the eager prefill is launch-bound.

    python tools/diag/prefill_small.py [--tokens 21] [--reps 10]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=21)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--dir", default=os.environ.get("NLS_BENCH_DIR", "/tmp/nls_bench"))
    ap.add_argument("--cprofile", action="store_true", help="host profile of the timed generate calls")
    a = ap.parse_args()
    from nats_llm_studio_amd.engine.engine import Engine
    from nats_llm_studio_amd.engine.sampling import SamplingParams
    from nats_llm_studio_amd.gguf.reader import GGUFReader
    from nats_llm_studio_amd.gguf.synth import write_synthetic_gguf
    from nats_llm_studio_amd.models.llama import LlamaModel
    path = os.path.join(a.dir, f"{a.model}-Q4_K_M.gguf")
    if not os.path.exists(path):
        os.makedirs(a.dir, exist_ok=True)
        write_synthetic_gguf(path, a.model, "Q4_K_M", seed=0)
    dev = torch.device("cuda:0")
    m = LlamaModel(GGUFReader(path), dev)
    eng = Engine(m, None, max_batch=8, ctx=1024)
    eng.capture_all()
    rec = []
    fwd = m.forward

    def timed_forward(*args, **kw):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        out = fwd(*args, **kw)
        t1 = time.perf_counter()
        e1.record()
        rec.append((args[3], t1 - t0, e0, e1))
        return out
    m.forward = timed_forward
    rng = np.random.default_rng(0)
    walls = []
    prof = None
    if a.cprofile:
        import cProfile
        prof = cProfile.Profile()
    for i in range(a.reps + 2):
        if prof is not None and i == 2:
            prof.enable()
        rec.clear()
        ids = [int(t) for t in rng.integers(10, 50000, a.tokens)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.generate(ids, SamplingParams(max_tokens=1, ignore_eos=True))
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        if i >= 2:
            for T, host, e0, e1 in rec:
                print(f"forward T={T}: host {host * 1e3:.3f} ms, gpu {e0.elapsed_time(e1):.3f} ms", flush=True)
    if prof is not None:
        prof.disable()
        import pstats
        pstats.Stats(prof).sort_stats("tottime").print_stats(30)
    w = sorted(walls[2:])
    print(f"generate({a.tokens} tokens, 1 new): wall p50 {w[len(w) // 2] * 1e3:.3f} ms", flush=True)
    print(f"engine host_ms {eng.host_ms}", flush=True)


if __name__ == "__main__":
    main()
