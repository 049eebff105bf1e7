"""Whole-model GPU tests: engine (HIP kernels + hipGraph decode) vs fp32 reference."""
import numpy as np
import pytest
import torch

from nats_llm_studio_amd.engine.engine import Engine, GenRequest
from nats_llm_studio_amd.engine.sampling import SamplingParams
from nats_llm_studio_amd.gguf.reader import GGUFReader
from nats_llm_studio_amd.models.llama import LlamaModel
from nats_llm_studio_amd.models.reference import ReferenceModel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral", "tiny-granite", "tiny-llama31", "tiny-qwen2"])
def test_prefill_logits_match_reference(gpu, tiny_models, name):
    r = GGUFReader(tiny_models[name])
    m = LlamaModel(r, gpu)
    ref = ReferenceModel(r)
    S = 40
    ids = list(np.random.default_rng(0).integers(0, 900, S))
    b = m.step_buffers(64, 4, 8)
    kc, vc = m.kv_cache(8, 16)
    b.ids[:S] = torch.tensor(ids, dtype=torch.int32)
    b.pos[:S] = torch.arange(S)
    b.slot[:S] = torch.arange(S)
    b.tok_seq[:S] = 0
    b.ctx_len[:S] = torch.arange(S) + 1
    b.block_tables[0] = torch.arange(8)
    m.forward(b, kc, vc, S, 16, n_split=2)
    rl = ref.logits(ids)
    err = (b.logits[:S].cpu() - rl).abs().max().item()
    assert err < 0.05 * rl.abs().max().item(), err
    agree = (b.next_ids[:S].cpu() == rl.argmax(1)).float().mean().item()
    assert agree > 0.9


@pytest.mark.parametrize("ft", ["Q4_0", "Q4_1", "Q5_0", "Q5_1", "Q3_K_M", "Q2_K"])
def test_new_quant_mixes_match_reference(gpu, tiny_ftypes, ft):
    """Whole models in the re-encoded mixes on the GPU kernels: prefill logits vs the fp32 oracle of the
    original GGUF bytes, then hipGraph decode == eager decode."""
    r = GGUFReader(tiny_ftypes[ft])
    m = LlamaModel(r, gpu)
    ref = ReferenceModel(r)
    S = 40
    ids = list(np.random.default_rng(0).integers(0, 900, S))
    b = m.step_buffers(64, 4, 8)
    kc, vc = m.kv_cache(8, 16)
    b.ids[:S] = torch.tensor(ids, dtype=torch.int32)
    b.pos[:S] = torch.arange(S)
    b.slot[:S] = torch.arange(S)
    b.tok_seq[:S] = 0
    b.ctx_len[:S] = torch.arange(S) + 1
    b.block_tables[0] = torch.arange(8)
    m.forward(b, kc, vc, S, 16, n_split=2)
    rl = ref.logits(ids)
    err = (b.logits[:S].cpu() - rl).abs().max().item()
    assert err < 0.05 * rl.abs().max().item(), err
    outs = []
    for graphs in (False, True):
        eng = Engine(m, None, max_batch=4, use_graphs=graphs)
        futs = [eng.submit(GenRequest([1, 2, 3, 4 + i], SamplingParams(max_tokens=8, ignore_eos=True)))
                for i in range(3)]
        while not all(f.done() for f in futs):
            eng.step()
        outs.append([f.result().token_ids for f in futs])
    assert outs[0] == outs[1]


def test_moe_grouped_gemm_prefill(gpu, tiny_models):
    """T > 64 routes every token at once and runs the experts as mapped-row LDS GEMMs (mode 2)."""
    r = GGUFReader(tiny_models["tiny-mixtral"])
    m = LlamaModel(r, gpu)
    ref = ReferenceModel(r)
    S, n = 150, 48
    ids = list(np.random.default_rng(1).integers(0, 900, S))
    b = m.step_buffers(256, 4, 16)
    kc, vc = m.kv_cache(16, 16)
    b.ids[:S] = torch.tensor(ids, dtype=torch.int32)
    b.pos[:S] = torch.arange(S)
    b.slot[:S] = torch.arange(S)
    b.tok_seq[:S] = 0
    b.ctx_len[:S] = torch.arange(S) + 1
    b.block_tables[0] = torch.arange(16)
    rows = torch.arange(S - n, S, dtype=torch.int32, device=gpu)
    m.forward(b, kc, vc, S, 16, n_split=2, logit_rows=rows, n_logits=n)
    rl = ref.logits(ids)[S - n:]
    err = (b.logits[:n].cpu() - rl).abs().max().item()
    assert err < 0.05 * rl.abs().max().item(), err


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral"])
@pytest.mark.parametrize("graphs", [False, True])
def test_engine_greedy_matches_reference(gpu, tiny_models, name, graphs):
    r = GGUFReader(tiny_models[name])
    m = LlamaModel(r, gpu)
    ref = ReferenceModel(r)
    eng = Engine(m, None, max_batch=8, max_prefill_tokens=48, use_graphs=graphs)
    rng = np.random.default_rng(1)
    prompts = [list(rng.integers(0, 900, n)) for n in (5, 17, 33, 50, 3)]
    futs = [eng.submit(GenRequest(p, SamplingParams(max_tokens=8, ignore_eos=True))) for p in prompts]
    while not all(f.done() for f in futs):
        eng.step()
    ok = 0
    for p, f in zip(prompts, futs):
        res = f.result()
        exp = ref.greedy(p, 8)
        ok += sum(int(a == b) for a, b in zip(res.token_ids, exp))
        assert res.token_ids[0] == exp[0]
    assert ok >= 0.85 * 8 * len(prompts)
    if graphs:
        assert eng.counters["graph_replays"] > 0


def test_engine_async_first_tokens_match_sync(gpu, tiny_models, monkeypatch):
    """The first tokens of finished prompts read back once per engine step (greedy ids and device-sampler draws
    behind an event, engine._ASYNC_FIRST) equal the per-chunk synchronous picks, greedy and seeded sampled."""
    from nats_llm_studio_amd.engine import engine as E
    r = GGUFReader(tiny_models["tiny-llama"])
    m = LlamaModel(r, gpu)
    rng = np.random.default_rng(3)
    prompts = [[int(t) for t in rng.integers(0, 900, n)] for n in (5, 40, 17, 90, 33, 8)]
    params = [SamplingParams(max_tokens=6, ignore_eos=True),
              SamplingParams(max_tokens=6, temperature=0.8, top_k=40, seed=1, ignore_eos=True),
              SamplingParams(max_tokens=6, temperature=1.1, top_p=0.9, repeat_penalty=1.2, seed=2, ignore_eos=True),
              SamplingParams(max_tokens=6, ignore_eos=True),
              SamplingParams(max_tokens=1, temperature=0.7, seed=3, ignore_eos=True),
              SamplingParams(max_tokens=6, temperature=0.9, min_p=0.05, seed=4, ignore_eos=True)]
    outs = []
    for flag in (False, True):
        monkeypatch.setattr(E, "_ASYNC_FIRST", flag)
        eng = Engine(m, None, max_batch=8, max_prefill_tokens=48, use_graphs=True)
        futs = [eng.submit(GenRequest(p, sp)) for p, sp in zip(prompts, params)]
        while not all(f.done() for f in futs):
            eng.step()
        outs.append([f.result().token_ids for f in futs])
        assert not eng._first_pending
    assert outs[0] == outs[1]


def test_engine_long_prompt_back_to_back_chunks(gpu, tiny_models):
    """A 300-token prompt at 32-token chunks: the engine queues several chunks per step with no token read back
    in between (a non_blocking upload from pinned memory reads the host buffer when it runs, so each chunk's
    metadata needs its own staging set), and the GPU is kept busy ahead of them so the uploads run late.
    The first tokens must equal the fp32 reference."""
    r = GGUFReader(tiny_models["tiny-llama"])
    m = LlamaModel(r, gpu)
    ref = ReferenceModel(r)
    eng = Engine(m, None, max_batch=4, max_prefill_tokens=32, use_graphs=False, ctx=512)
    rng = np.random.default_rng(7)
    p = [int(t) for t in rng.integers(0, 900, 300)]
    x = torch.randn(4096, 4096, device=gpu, dtype=torch.float16)
    for _ in range(8):                       # queued GPU work ahead of the first chunk's uploads
        x = x @ x.t() * 1e-4
    fut = eng.submit(GenRequest(p, SamplingParams(max_tokens=4, ignore_eos=True)))
    while not fut.done():
        eng.step()
    exp = ref.greedy(p, 4)
    got = fut.result().token_ids
    assert got[0] == exp[0], (got, exp)
    assert sum(int(a == b) for a, b in zip(got, exp)) >= 3, (got, exp)


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral"])
def test_engine_fp8_kv_cache(gpu, tiny_models, name, monkeypatch):
    """NLS_KV_DTYPE=fp8: an OCP e4m3 paged KV cache (half the attention bytes) through prefill (MFMA flash
    prefill), the graph-captured decode and the fused RoPE/KV-append paths; greedy tokens stay close to
    the fp32 reference (e4m3 rounds K/V to 3 mantissa bits, so exact agreement is not expected)."""
    monkeypatch.setenv("NLS_KV_DTYPE", "fp8")
    r = GGUFReader(tiny_models[name])
    m = LlamaModel(r, gpu)
    ref = ReferenceModel(r)
    eng = Engine(m, None, max_batch=8, max_prefill_tokens=48, use_graphs=True)
    assert eng.kc.dtype == torch.float8_e4m3fn
    rng = np.random.default_rng(2)
    prompts = [list(rng.integers(0, 900, n)) for n in (5, 17, 33, 50, 3)]
    futs = [eng.submit(GenRequest(p, SamplingParams(max_tokens=8, ignore_eos=True))) for p in prompts]
    while not all(f.done() for f in futs):
        eng.step()
    ok = sum(sum(int(a == b) for a, b in zip(f.result().token_ids, ref.greedy(p, 8))) for p, f in zip(prompts, futs))
    assert ok >= 0.7 * 8 * len(prompts), ok
    assert eng.counters["graph_replays"] > 0


@pytest.mark.parametrize("precapture", [False, True])
def test_prefill_graphs_match_eager(gpu, tiny_models, monkeypatch, precapture):
    """Single-prompt prefill chunks of <= 64 tokens replay a captured graph of their token bucket (16 / 32 / 64;
    padded rows write no KV and are never read): greedy and seeded-sampled tokens equal the eager prefill, the
    first greedy token equals the fp32 reference, and a second prompt of a bucket replays its graph."""
    from nats_llm_studio_amd.engine import engine as E
    r = GGUFReader(tiny_models["tiny-llama"])
    m = LlamaModel(r, gpu)
    ref = ReferenceModel(r)
    rng = np.random.default_rng(11)
    lens = (5, 16, 17, 33, 64, 65, 9, 30)
    prompts = [[int(t) for t in rng.integers(0, 900, n)] for n in lens]
    params = [SamplingParams(max_tokens=5, ignore_eos=True) if i % 2 == 0 else
              SamplingParams(max_tokens=5, temperature=0.8, top_k=20, seed=i, ignore_eos=True) for i in range(len(lens))]
    outs, counters = [], []
    for flag in (False, True):
        monkeypatch.setattr(E, "_PREFILL_GRAPHS", flag)
        eng = Engine(m, None, max_batch=4, max_prefill_tokens=128, use_graphs=True)
        if precapture:
            eng.capture_all()
        res = []
        for p, sp in zip(prompts, params):           # one prompt at a time: each prefill is its own chunk
            f = eng.submit(GenRequest(list(p), sp))
            while not f.done():
                eng.step()
            res.append(f.result().token_ids)
        outs.append(res)
        counters.append(dict(eng.counters))
    assert outs[0] == outs[1]
    assert counters[0]["prefill_graph_replays"] == 0
    # keys (bucket 16 / 32 / 64, logits): lazily, only the 9-token greedy prompt finds its (16, greedy) graph; precaptured, all 7 <= 64 do
    assert counters[1]["prefill_graph_replays"] >= (7 if precapture else 1), counters[1]
    for p, sp, toks in zip(prompts, params, outs[1]):
        if sp.greedy:
            assert toks[0] == ref.greedy(p, 1)[0]


def test_graph_equals_eager(gpu, tiny_models):
    r = GGUFReader(tiny_models["tiny-llama"])
    m = LlamaModel(r, gpu)
    outs = []
    for graphs in (False, True):
        eng = Engine(m, None, max_batch=4, use_graphs=graphs)
        futs = [eng.submit(GenRequest([1, 2, 3, 4 + i], SamplingParams(max_tokens=12, ignore_eos=True)))
                for i in range(3)]
        while not all(f.done() for f in futs):
            eng.step()
        outs.append([f.result().token_ids for f in futs])
    assert outs[0] == outs[1]


def test_device_sampling_in_graph(gpu, tiny_models):
    """Sampled rows stay on the chained decode graph (ops.sample_decode): top_k=1 sampling equals
    greedy, seeded draws reproduce, and the device penalty window (history ring filled at row
    assignment, appended in-graph) bans every recent token under a huge presence penalty."""
    r = GGUFReader(tiny_models["tiny-llama"])
    m = LlamaModel(r, gpu)
    prompt = [5, 17, 99, 3, 250, 7, 81, 12]

    def run(params_list):
        eng = Engine(m, None, max_batch=8, use_graphs=True)
        futs = [eng.submit(GenRequest(list(prompt), p)) for p in params_list]
        while not all(f.done() for f in futs):
            eng.step()
        return [f.result().token_ids for f in futs], eng.counters["device_sampled_steps"]

    g = SamplingParams(max_tokens=12, ignore_eos=True)
    k1 = SamplingParams(max_tokens=12, ignore_eos=True, temperature=1.0, top_k=1)
    (a, b), n = run([g, k1])
    assert a == b and n > 0
    s1 = SamplingParams(max_tokens=12, ignore_eos=True, temperature=1.5, seed=11)
    s2 = SamplingParams(max_tokens=12, ignore_eos=True, temperature=1.5, seed=12)
    (x1, y1), _ = run([s1, s2])
    (x2, y2), _ = run([s1, s2])
    assert x1 == x2 and y1 == y2
    ban = SamplingParams(max_tokens=20, ignore_eos=True, temperature=1.0, top_k=1, presence_penalty=1e9)
    (t,), _ = run([ban])
    assert len(set(t)) == len(t) and not (set(t[1:]) & set(prompt)), t


@pytest.mark.parametrize("graphs", [False, True])
def test_split_rmsnorm_decode_matches_plain(gpu, tiny_models, graphs):
    """Few-row decode with every RMSNorm split between the O/down GEMVs (shares of sum(x^2)) and the
    consuming GEMVs == the plain path with norm launches, token for token."""
    from nats_llm_studio_amd.engine.engine import Engine, GenRequest
    from nats_llm_studio_amd.engine.sampling import SamplingParams
    from nats_llm_studio_amd.gguf.reader import GGUFReader
    from nats_llm_studio_amd.models.llama import LlamaModel
    r = GGUFReader(tiny_models["tiny-llama"])
    outs = []
    for fuse in (False, True):
        m = LlamaModel(r, gpu, fuse_norm=fuse)
        eng = Engine(m, None, max_batch=4, num_blocks=64, use_graphs=graphs, ctx=256)
        futs = [eng.submit(GenRequest([1, 2, 3, 40 + i], SamplingParams(max_tokens=12, ignore_eos=True)))
                for i in range(3)]
        while not all(f.done() for f in futs):
            eng.step()
        outs.append([f.result().token_ids for f in futs])
        eng.shutdown()
    agree = sum(int(a == b) for r0, r1 in zip(*outs) for a, b in zip(r0, r1))
    assert outs[0][0][:4] == outs[1][0][:4] and agree >= 30, outs


def test_seeded_sampling_same_on_device_and_host_paths(gpu, tiny_models, monkeypatch):
    """A seeded request draws u = uniform01(seed, position) on every path: the in-graph sampler
    (chained decode) and the host-driven batched GPU sampler (NLS_DEVICE_SAMPLING=0, the path tensor
    parallel and logits requests take) produce the same tokens for the same seeds."""
    r = GGUFReader(tiny_models["tiny-llama"])
    m = LlamaModel(r, gpu)
    prompt = [5, 17, 99, 3, 250, 7, 81, 12]
    ps = [SamplingParams(max_tokens=16, ignore_eos=True, temperature=1.3, top_p=0.95, top_k=40, seed=s)
          for s in (3, 4, 5)]

    def run(dev):
        monkeypatch.setenv("NLS_DEVICE_SAMPLING", "1" if dev else "0")
        eng = Engine(m, None, max_batch=4, use_graphs=True)
        assert eng.device_sampling == dev
        futs = [eng.submit(GenRequest(list(prompt), p)) for p in ps]
        while not all(f.done() for f in futs):
            eng.step()
        return [f.result().token_ids for f in futs], eng.counters["device_sampled_steps"]
    a, na = run(True)
    b, nb = run(False)
    assert na > 0 and nb == 0
    assert a == b, (a, b)


@pytest.mark.parametrize("graphs", [False, True])
def test_moe_folded_route_matches_separate_launch(gpu, tiny_models, graphs, monkeypatch):
    """MoE decode at <= 4 tokens: the FFN norm + router + top-k route in the o projection's last workgroup
    (ops.qgemv_add_norm_route) == the separate moe_norm_route launch, token for token (both multiply the same
    f16 normalised rows with the router's f16 copy)."""
    from nats_llm_studio_amd.engine.engine import Engine, GenRequest
    from nats_llm_studio_amd.engine.sampling import SamplingParams
    from nats_llm_studio_amd.gguf.reader import GGUFReader
    from nats_llm_studio_amd.models import llama
    r = GGUFReader(tiny_models["tiny-mixtral"])
    outs = []
    for fold in (False, True):
        monkeypatch.setattr(llama, "_MOE_FOLD_ROUTE", fold)
        m = llama.LlamaModel(r, gpu)
        eng = Engine(m, None, max_batch=4, num_blocks=64, use_graphs=graphs, ctx=256)
        futs = [eng.submit(GenRequest([1, 2, 3, 40 + i], SamplingParams(max_tokens=12, ignore_eos=True)))
                for i in range(3)]
        while not all(f.done() for f in futs):
            eng.step()
        outs.append([f.result().token_ids for f in futs])
        eng.shutdown()
    assert outs[0] == outs[1], outs
