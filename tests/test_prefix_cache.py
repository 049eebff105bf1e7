"""Automatic prefix caching: shared prompt prefixes reuse KV blocks (CPU engine, same code as GPU)."""
import numpy as np

from nats_llm_studio_amd.engine.engine import BlockAllocator, Engine, GenRequest
from nats_llm_studio_amd.engine.sampling import SamplingParams
from nats_llm_studio_amd.gguf.reader import GGUFReader
from nats_llm_studio_amd.models.llama import LlamaModel


def _run(eng, prompts, n=6):
    futs = [eng.submit(GenRequest(list(p), SamplingParams(max_tokens=n, ignore_eos=True))) for p in prompts]
    while not all(f.done() for f in futs):
        eng.step()
    return [f.result().token_ids for f in futs]


def test_allocator_refcount_lru_eviction():
    a = BlockAllocator(4)
    keys = BlockAllocator.chain_keys(list(range(64)), 16, 3)
    b1 = a.alloc(3)
    a.register(b1, keys)
    a.release(b1)                        # cached, ref 0 -> LRU (still matchable)
    assert a.n_free == 4
    hit = a.match(keys[:2])
    assert hit == b1[:2] and a.n_free == 2
    more = a.alloc(2)                    # 1 never-used block + evicts the LRU cached block b1[2]
    assert b1[2] in more and keys[2] not in a.block_of
    assert a.alloc(1) is None
    a.release(hit + more)
    assert a.n_free == 4


def test_prefix_cache_hits_and_identical_outputs(tiny_models):
    r = GGUFReader(tiny_models["tiny-llama"])
    m = LlamaModel(r, "cpu")
    rng = np.random.default_rng(3)
    system = list(rng.integers(0, 900, 40))              # shared "system prompt" (2 full blocks + 8)
    prompts = [system + list(rng.integers(0, 900, k)) for k in (5, 11, 23)]
    ref = _run(Engine(m, None, max_batch=4, num_blocks=64, use_graphs=False, ctx=256, prefix_cache=False),
               prompts)
    eng = Engine(m, None, max_batch=4, num_blocks=64, use_graphs=False, ctx=256)
    first = _run(eng, prompts[:1])
    assert eng.stats()["prefix_cache_hit_tokens"] == 0
    rest = _run(eng, prompts[1:])
    assert first + rest == ref
    assert eng.stats()["prefix_cache_hit_tokens"] == 2 * 32     # two later requests x 2 cached blocks
    assert eng.stats()["kv_blocks_free"] == 64
