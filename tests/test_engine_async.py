"""Chained (async) decode == synchronous decode on CPU: stable rows, next-token chaining through
`use_prev`, stop conditions that are only known one step late (stop ids / EOS), max_tokens
budgets, staggered admissions and row compaction."""
import pytest
import torch

from nats_llm_studio_amd.engine.engine import Engine, GenRequest
from nats_llm_studio_amd.engine.sampling import SamplingParams
from nats_llm_studio_amd.gguf.reader import GGUFReader
from nats_llm_studio_amd.models.llama import LlamaModel


def _engine(path, async_decode):
    m = LlamaModel(GGUFReader(path), "cpu")
    return Engine(m, None, max_batch=8, max_prefill_tokens=64, num_blocks=128, use_graphs=False, ctx=256,
                  async_decode=async_decode)


def _run(eng, reqs, stagger):
    futs = []
    pending = list(reqs)
    steps = 0
    while pending or not all(f.done() for f in futs):
        if pending and steps % stagger == 0:
            futs.append(eng.submit(GenRequest(*pending.pop(0))))
        eng.step()
        steps += 1
        assert steps < 2000
    return [(f.result().token_ids, f.result().finish_reason, f.result().stop_reason) for f in futs]


@pytest.mark.parametrize("stagger", [1, 3])
def test_async_matches_sync(tiny_models, stagger):
    path = tiny_models["tiny-llama"]
    base = _run(_engine(path, False), [([1, 2, 3, 4, 5], SamplingParams(max_tokens=12, ignore_eos=True))], 1)
    stop_tok = base[0][0][4]                      # the 5th greedy token: an early, data-dependent stop
    reqs = [
        ([1, 2, 3, 4, 5], SamplingParams(max_tokens=12, ignore_eos=True)),
        ([1, 2, 3, 4, 5], SamplingParams(max_tokens=12, ignore_eos=True, stop_token_ids=[stop_tok])),
        ([9, 8, 7], SamplingParams(max_tokens=1, ignore_eos=True)),
        ([9, 8, 7, 6, 5, 4, 3, 2, 1, 11, 12, 13, 14, 15, 16, 17, 18], SamplingParams(max_tokens=20, ignore_eos=True)),
        ([42] * 30, SamplingParams(max_tokens=7, ignore_eos=True)),
        ([5, 6], SamplingParams(max_tokens=3, ignore_eos=True)),
    ]
    sync = _run(_engine(path, False), reqs, stagger)
    eng = _engine(path, True)
    asyn = _run(eng, reqs, stagger)
    assert asyn == sync
    assert sync[1][2] == "stopTokenFound" and len(sync[1][0]) == 5
    assert all(r is None for r in eng.rows) and eng._inflight is None
    assert eng.alloc.n_free == eng.num_blocks
