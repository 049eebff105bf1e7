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


@pytest.mark.parametrize("ft", ["Q4_0", "Q4_1", "Q5_0", "Q5_1", "Q3_K_M", "Q2_K"])
def test_cpu_prefill_new_quant_mixes(tiny_ftypes, ft):
    """GGUF mixes of the legacy 32-block types and the low-bit K types load (the weights re-encoded for
    the device, ops/transcode.py; the CPU path decodes the original bytes) and match the oracle; the
    registry-facing file_type round-trips."""
    from nats_llm_studio_amd.gguf.constants import FILE_TYPE_NAMES
    r = GGUFReader(tiny_ftypes[ft])
    assert FILE_TYPE_NAMES[int(r.metadata["general.file_type"])] == ft
    m = LlamaModel(r, "cpu")
    ref = ReferenceModel(r)
    S = 20
    ids = list(np.random.default_rng(1).integers(0, 900, S))
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


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral"])
def test_cpu_fp8_kv_cache_engine(tiny_models, name, monkeypatch):
    """NLS_KV_DTYPE=fp8: the paged KV cache is OCP e4m3 (the CPU reference paths round through the same
    dtype); greedy decoding still tracks the fp32 reference closely."""
    from nats_llm_studio_amd.engine.engine import Engine, GenRequest
    from nats_llm_studio_amd.engine.sampling import SamplingParams
    monkeypatch.setenv("NLS_KV_DTYPE", "fp8")
    r = GGUFReader(tiny_models[name])
    m = LlamaModel(r, "cpu")
    ref = ReferenceModel(r)
    eng = Engine(m, None, max_batch=4, max_prefill_tokens=32, use_graphs=False)
    assert eng.kc.dtype == torch.float8_e4m3fn
    prompts = [[5, 9, 200, 33], list(range(40, 60))]
    futs = [eng.submit(GenRequest(p, SamplingParams(max_tokens=6, ignore_eos=True))) for p in prompts]
    while not all(f.done() for f in futs):
        eng.step()
    ok = sum(sum(int(a == b) for a, b in zip(f.result().token_ids, ref.greedy(p, 6))) for p, f in zip(prompts, futs))
    assert ok >= 0.6 * 12, ok
    monkeypatch.setenv("NLS_KV_DTYPE", "fp16")
    with pytest.raises(ValueError):
        m.kv_cache(2, 16)


def test_cpu_moe_norm_route_reference():
    """ops.moe_norm_route on CPU == rmsnorm, then h @ Wr^T, then the top-k route."""
    from nats_llm_studio_amd import ops
    g = torch.Generator().manual_seed(3)
    T, D, E, k, cap = 3, 256, 8, 2, 8
    x = torch.randn(cap, D, generator=g)
    nw = torch.rand(D, generator=g) + 0.5
    wr = (torch.randn(E, D, generator=g) * 0.1).half()
    bufs = [dict(h=torch.zeros(cap, D, dtype=ops.ACT_DTYPE), lg=torch.zeros(cap, E), topw=torch.zeros(cap * k),
                 counts=torch.zeros(E, dtype=torch.int32), xr=torch.zeros(E * cap, dtype=torch.int32),
                 yr=torch.zeros(E * cap, dtype=torch.int32)) for _ in range(2)]
    a, b = bufs
    assert ops.moe_norm_route(x, nw, 1e-5, wr, a["h"], a["lg"], T, k, a["topw"], a["counts"], a["xr"], a["yr"], cap)
    ops.rmsnorm(x, nw, b["h"], T, 1e-5)
    b["lg"][:T] = b["h"][:T].float() @ wr.float().t()
    ops.moe_route(b["lg"], T, k, b["topw"], b["counts"], b["xr"], b["yr"], cap)
    for key in a:
        assert torch.equal(a[key], b[key]), key


def test_reference_streaming_decode_matches_cached(tiny_models):
    """The oracle's streaming mode (cache=False, parallel row-range decoding, gathered embedding rows)
    computes exactly what the cached whole-tensor mode does."""
    from nats_llm_studio_amd.gguf.reader import GGUFReader
    from nats_llm_studio_amd.models.reference import ReferenceModel
    for name in ("tiny-llama", "tiny-mixtral"):
        r = GGUFReader(tiny_models[name])
        ids = [1, 5, 9, 200, 33, 7]
        a = ReferenceModel(r).logits(ids)
        b = ReferenceModel(r, cache=False, workers=4).logits(ids)
        assert torch.equal(a, b)


def test_tuning_role_fallback_scope(monkeypatch):
    """Untuned few-row shapes within 1.5x of a Llama-3-8B projection (Qwen2.5-7B) borrow that role's tuned
    entry; larger shapes (Llama-3-70B) keep the generic heuristic; NLS_TUNING_ROLE=0 turns borrowing off;
    an exact table entry always wins (ops/tuning.py select)."""
    from types import SimpleNamespace as N
    from nats_llm_studio_amd.ops import tuning

    def segs(*parts):
        return [N(w=N(type=t, rows=r, K=k)) for t, r, k in parts]

    tab = tuning.table()
    qwen_gu, qwen_qkv = segs((12, 37888, 3584)), segs((12, 3584, 3584), (12, 512, 3584), (12, 512, 3584))
    l70_o = segs((12, 8192, 8192))
    for M in (16, 64):
        assert tuning.key(qwen_gu, M) not in tab
        assert tuning._role(qwen_gu) == "gateup" and tuning._role(qwen_qkv) == "qkv" and tuning._role(l70_o) == "o"
        assert tuning.select(qwen_gu, M) == tab[f"12:28672:4096:{M}"]
        assert tuning.select(qwen_qkv, M) == tab[f"12+12+12:6144:4096:{M}"]
        assert tuning._role_entry(l70_o, M) is None
        assert tuning.select(l70_o, M) == tuning.heuristic(l70_o, M)
    monkeypatch.setenv("NLS_TUNING_ROLE", "0")
    assert tuning.select(qwen_gu, 16) == tuning.heuristic(qwen_gu, 16)
    monkeypatch.setitem(tab, tuning.key(qwen_gu, 16), (0, 4, 1, 1))
    assert tuning.select(qwen_gu, 16) == (0, 4, 1, 1)


def test_dense_segment_merge():
    """Dense launches see one segment per run of f16 copies that are consecutive rows of one buffer with adjacent
    output columns (a layer's Q|K|V after QWeight.expand_dense_group); separate buffers, gaps in the output columns
    and mapped (MoE) segments stay apart."""
    from types import SimpleNamespace as NS
    from nats_llm_studio_amd import ops
    K = 64
    buf = torch.zeros(96 + 32 + 32, K, dtype=torch.float16)
    q, k, v = (NS(name=n, rows=r, K=K, d16=buf[a:a + r]) for n, r, a in (("q", 96, 0), ("k", 32, 96), ("v", 32, 128)))
    m = ops._merge_dense([ops.Seg(q, 0), ops.Seg(k, 96), ops.Seg(v, 128)])
    assert [(x[0], x[1], x[3]) for x in m] == [(buf.data_ptr(), 160, 0)]
    other = NS(name="o", rows=32, K=K, d16=torch.zeros(32, K, dtype=torch.float16))
    m = ops._merge_dense([ops.Seg(q, 0), ops.Seg(k, 96), ops.Seg(other, 128)])
    assert [x[1] for x in m] == [128, 32]
    m = ops._merge_dense([ops.Seg(q, 0), ops.Seg(k, 100)])            # output columns not adjacent
    assert [x[1] for x in m] == [96, 32]
    xm = torch.zeros(4, dtype=torch.int32)
    m = ops._merge_dense([ops.Seg(q, 0, xm, xm), ops.Seg(k, 96, xm, xm)])
    assert [x[1] for x in m] == [96, 32] and m[1][4].xmap is xm
    with pytest.raises(ValueError):
        ops._merge_dense([ops.Seg(NS(name="n", rows=8, K=K, d16=None), 0)])


def test_tuning_extra_overrides(monkeypatch, tmp_path):
    """A/B overrides on top of ops/gemv_tuning.json: NLS_TUNING_EXTRA_FILE (a tune_gemv.py --out table) applies first,
    NLS_TUNING_EXTRA (inline JSON) over it; the table reloads with them and without them."""
    import json
    from nats_llm_studio_amd.ops import tuning
    key = "d:6144:4096:512"
    f = tmp_path / "extra.json"
    f.write_text(json.dumps({key: [4, 8, 2, 3], "d:1:2:3": [-1]}))
    monkeypatch.setattr(tuning, "_TABLE", None)
    base = dict(tuning.table())
    try:
        monkeypatch.setattr(tuning, "_TABLE", None)
        monkeypatch.setenv("NLS_TUNING_EXTRA_FILE", str(f))
        t = tuning.table()
        assert t[key] == (4, 8, 2, 3) and t["d:1:2:3"] == (-1,)
        monkeypatch.setattr(tuning, "_TABLE", None)
        monkeypatch.setenv("NLS_TUNING_EXTRA", json.dumps({key: [10, 8, 2, 1]}))
        t = tuning.table()
        assert t[key] == (10, 8, 2, 1) and t["d:1:2:3"] == (-1,)
        assert {k: v for k, v in t.items() if k not in (key, "d:1:2:3")} == {k: v for k, v in base.items() if k != key}
    finally:
        monkeypatch.delenv("NLS_TUNING_EXTRA_FILE", raising=False)
        monkeypatch.delenv("NLS_TUNING_EXTRA", raising=False)
        monkeypatch.setattr(tuning, "_TABLE", None)
