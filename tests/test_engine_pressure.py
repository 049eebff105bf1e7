"""KV-pool pressure on CPU: more concurrent requests than the block pool holds, so admissions wait
for finished sequences, freed blocks are reused and cached prefix blocks are evicted, all while
decode steps are chained asynchronously. Every request must produce exactly the tokens it
produces on an engine with room to spare (greedy decode is deterministic), and the pool must come
back whole. Rows are batched differently in the two engines, so CPU matmul rounding can differ in
the last bits: a divergence is accepted only where the reference's top-2 logit margin is a tie
(< 1e-3, checked by a single-sequence forward of the common prefix)."""
import numpy as np

from nats_llm_studio_amd.engine.engine import Engine, GenRequest
from nats_llm_studio_amd.engine.sampling import SamplingParams
from nats_llm_studio_amd.gguf.reader import GGUFReader
from nats_llm_studio_amd.models.llama import LlamaModel


def _reqs(n=24, seed=3):
    rng = np.random.default_rng(seed)
    system = [7, 3, 9, 11, 2, 5, 8, 13, 21, 4, 6, 10, 12, 14, 15, 16, 17, 18]   # shared prefix: cache hits
    out = []
    for i in range(n):
        tail = [int(v) for v in rng.integers(20, 200, int(rng.integers(1, 12)))]
        out.append((system + tail if i % 3 else tail, SamplingParams(max_tokens=int(rng.integers(1, 24)),
                                                                     ignore_eos=True)))
    return out


def _run_all(eng, reqs):
    futs = [eng.submit(GenRequest(list(t), p)) for t, p in reqs]
    steps = 0
    while not all(f.done() for f in futs):
        eng.step()
        steps += 1
        assert steps < 5000
    return [f.result().token_ids for f in futs]


def _margin(m, tokens):
    """Top-2 logit margin after `tokens` (single-sequence prefill; a sampled request materialises logits)."""
    eng = Engine(m, None, max_batch=1, max_prefill_tokens=128, num_blocks=16, use_graphs=False, ctx=128)
    eng.submit(GenRequest(list(tokens), SamplingParams(max_tokens=1, ignore_eos=True, temperature=1.0, seed=1)))
    eng.step()
    v = eng.pb.logits[0].float().topk(2).values
    return float(v[0] - v[1])


def test_pool_pressure_matches_roomy_engine(tiny_models):
    m = LlamaModel(GGUFReader(tiny_models["tiny-llama"]), "cpu")
    reqs = _reqs()
    roomy = Engine(m, None, max_batch=32, max_prefill_tokens=64, num_blocks=512, use_graphs=False, ctx=128,
                   async_decode=False)
    ref = _run_all(roomy, reqs)
    # ~3 blocks per request (block 16): 12 blocks hold about 4 requests at a time
    tight = Engine(m, None, max_batch=8, max_prefill_tokens=24, num_blocks=12, use_graphs=False, ctx=128,
                   async_decode=True)
    got = _run_all(tight, reqs)
    for (t, p), a, b in zip(reqs, got, ref):
        assert len(a) == len(b) == p.max_tokens
        k = next((i for i in range(len(a)) if a[i] != b[i]), None)
        if k is not None:
            assert _margin(m, list(t) + b[:k]) < 1e-3, (a, b)
    assert tight.alloc.n_free == tight.num_blocks and all(r == 0 for r in tight.alloc.ref)
    assert tight._inflight is None and all(r is None for r in tight.rows)
