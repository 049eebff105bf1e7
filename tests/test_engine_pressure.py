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


def _run_all_pinned(eng, reqs, ratio):
    """_run_all with the admission estimate held at `ratio` (finished requests would otherwise raise it)."""
    futs = [eng.submit(GenRequest(list(t), p)) for t, p in reqs]
    steps = 0
    while not all(f.done() for f in futs):
        eng.gen_ratio = ratio
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


def test_preemption_completes_requests_larger_than_pool(tiny_models):
    """KV blocks are allocated as sequences grow: requests whose prompt + max_tokens together need
    ~2.5x the pool all run, the pool runs dry mid-decode, the most recently submitted sequences are
    preempted (blocks freed) and re-prefilled from prompt + generated tokens later, and every request
    still returns exactly max_tokens tokens -- the same tokens as on an engine with room to spare."""
    m = LlamaModel(GGUFReader(tiny_models["tiny-llama"]), "cpu")
    rng = np.random.default_rng(11)
    reqs = [([int(v) for v in rng.integers(20, 200, int(rng.integers(4, 14)))],
             SamplingParams(max_tokens=int(rng.integers(60, 100)), ignore_eos=True)) for _ in range(6)]
    roomy = Engine(m, None, max_batch=8, max_prefill_tokens=64, num_blocks=256, use_graphs=False, ctx=256,
                   async_decode=False)
    ref = _run_all(roomy, reqs)
    assert roomy.counters["preemptions"] == 0
    # 16 blocks x 16 = 256 token slots for ~6 x 95 tokens of KV
    tight = Engine(m, None, max_batch=8, max_prefill_tokens=32, num_blocks=16, use_graphs=False, ctx=256,
                   async_decode=True)
    # as if earlier requests had stopped early: expected-growth admission is as optimistic as on-demand
    tight.gen_ratio = 0.05
    got = _run_all_pinned(tight, reqs, 0.05)
    assert tight.counters["preemptions"] > 0, tight.stats()
    for (t, p), a, b in zip(reqs, got, ref):
        assert len(a) == len(b) == p.max_tokens
        k = next((i for i in range(len(a)) if a[i] != b[i]), None)
        if k is not None:
            assert _margin(m, list(t) + b[:k]) < 1e-3, (a, b)
    assert tight.alloc.n_free == tight.num_blocks and all(r == 0 for r in tight.alloc.ref)
    assert tight._inflight is None and all(r is None for r in tight.rows)


def test_full_reservation_mode_never_preempts(tiny_models, monkeypatch):
    monkeypatch.setenv("NLS_KV_RESERVE", "full")
    m = LlamaModel(GGUFReader(tiny_models["tiny-llama"]), "cpu")
    reqs = _reqs(n=10, seed=5)
    eng = Engine(m, None, max_batch=8, max_prefill_tokens=24, num_blocks=12, use_graphs=False, ctx=128)
    got = _run_all(eng, reqs)
    assert eng.counters["preemptions"] == 0 and eng.stats()["kv_reserve"] == "full"
    assert [len(g) for g in got] == [p.max_tokens for _, p in reqs]


def test_expected_growth_admission_avoids_thrash(tiny_models):
    """The same oversubscribed workload with the admission estimate learnt from completions (every request
    runs to max_tokens, so the ratio stays at 1): sequences wait for room instead of being admitted and
    preempted, nothing is recomputed, and the tokens are the roomy engine's."""
    m = LlamaModel(GGUFReader(tiny_models["tiny-llama"]), "cpu")
    rng = np.random.default_rng(11)
    reqs = [([int(v) for v in rng.integers(20, 200, int(rng.integers(4, 14)))],
             SamplingParams(max_tokens=int(rng.integers(60, 100)), ignore_eos=True)) for _ in range(6)]
    roomy = Engine(m, None, max_batch=8, max_prefill_tokens=64, num_blocks=256, use_graphs=False, ctx=256,
                   async_decode=False)
    ref = _run_all(roomy, reqs)
    tight = Engine(m, None, max_batch=8, max_prefill_tokens=32, num_blocks=16, use_graphs=False, ctx=256,
                   async_decode=True)
    got = _run_all(tight, reqs)
    assert tight.counters["preemptions"] == 0 and tight.counters["recompute_tokens"] == 0, tight.stats()
    assert tight.gen_ratio > 0.99
    for (t, p), a, b in zip(reqs, got, ref):
        assert len(a) == len(b) == p.max_tokens
        k = next((i for i in range(len(a)) if a[i] != b[i]), None)
        if k is not None:
            assert _margin(m, list(t) + b[:k]) < 1e-3, (a, b)
    assert tight.alloc.n_free == tight.num_blocks
