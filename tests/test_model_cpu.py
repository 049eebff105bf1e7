"""Whole-model CPU path (torch reference ops behind the same LlamaModel/Engine code the GPU runs)
vs the independent fp32 oracle (models/reference.py), incl. Llama-3.1 `rope_freqs` frequency factors."""
import numpy as np
import pytest
import torch

from nats_llm_studio_amd.gguf.reader import GGUFReader
from nats_llm_studio_amd.models.llama import LlamaModel
from nats_llm_studio_amd.models.reference import ReferenceModel


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-llama31", "tiny-granite", "tiny-qwen2"])
def test_cpu_prefill_matches_reference(tiny_models, name):
    r = GGUFReader(tiny_models[name])
    m = LlamaModel(r, "cpu")
    ref = ReferenceModel(r)
    S = 24
    ids = list(np.random.default_rng(0).integers(0, 900, S))
    b = m.step_buffers(64, 4, 8)
    kc, vc = m.kv_cache(8, 16)
    b.ids[:S] = torch.tensor(ids, dtype=torch.int32)
    b.pos[:S] = torch.arange(S)
    b.slot[:S] = torch.arange(S)
    b.tok_seq[:S] = 0
    b.ctx_len[:S] = torch.arange(S) + 1
    b.block_tables[0] = torch.arange(8)
    m.forward(b, kc, vc, S, 16)
    rl = ref.logits(ids)
    err = (b.logits[:S] - rl).abs().max().item()
    assert err < 0.02 * rl.abs().max().item(), err


def test_rope_freqs_change_the_rotation(tiny_models):
    """The Llama-3.1 factors are applied (a model that ignored them would differ from the oracle)."""
    from nats_llm_studio_amd import ops
    r = GGUFReader(tiny_models["tiny-llama31"])
    ff = r.dequantized("rope_freqs.weight")
    assert ff.max() > 1.0
    m = LlamaModel(r, "cpu")
    plain = ops.rope_table(m.cfg.ctx, m.D, m.cfg.rope_base, "cpu")
    assert not torch.allclose(m.cs[100], plain[100])


def test_fused_norm_decode_matches_unfused(tiny_models):
    """Few-row decode with the RMSNorms folded into the GEMVs (NLS_FUSE_NORM) == the plain path."""
    from nats_llm_studio_amd.engine.engine import Engine, GenRequest
    from nats_llm_studio_amd.engine.sampling import SamplingParams
    r = GGUFReader(tiny_models["tiny-llama"])
    outs = []
    for fuse in (False, True):
        m = LlamaModel(r, "cpu", fuse_norm=fuse)
        eng = Engine(m, None, max_batch=4, num_blocks=32, use_graphs=False, ctx=256)
        futs = [eng.submit(GenRequest([1, 2, 3, 40 + i], SamplingParams(max_tokens=6, ignore_eos=True)))
                for i in range(3)]
        while not all(f.done() for f in futs):
            eng.step()
        outs.append([f.result().token_ids for f in futs])
    assert outs[0] == outs[1]


def test_stop_strings_incremental(tiny_models):
    """A stop string that appears mid-generation ends the request there (stopStringFound) and is cut
    from the text; the check is incremental (stream decoder tail), not a re-decode per token."""
    from nats_llm_studio_amd.engine.engine import Engine, GenRequest
    from nats_llm_studio_amd.engine.sampling import SamplingParams
    from nats_llm_studio_amd.tokenizer.bpe import tokenizer_from_metadata
    r = GGUFReader(tiny_models["tiny-llama"])
    tok = tokenizer_from_metadata(r.metadata)
    m = LlamaModel(r, "cpu")
    eng = Engine(m, tok, max_batch=2, num_blocks=32, use_graphs=False, ctx=256)
    prompt = [1, 2, 3, 40]
    full = eng.generate(prompt, SamplingParams(max_tokens=24, ignore_eos=True))
    text = full.text
    assert len(text) > 8
    # a stop string taken from the middle of the generated text
    cut = len(tok.decode(full.token_ids[:8]))
    stop = text[cut:cut + 3]
    assert stop and stop in text
    first = text.find(stop)
    res = eng.generate(prompt, SamplingParams(max_tokens=24, ignore_eos=True, stop=[stop]))
    assert res.finish_reason == "stop" and res.stop_reason == "stopStringFound"
    assert res.text == text[:first]
    assert len(res.token_ids) < len(full.token_ids)
