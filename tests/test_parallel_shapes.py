"""Tensor / expert parallel rehearsals at the per-rank SHAPES of the north-star multi-GPU configs, on
CPU over gloo (the same sharding + comm + engine code the GPU path runs over RCCL / the one-shot IPC
all-reduce):

* Llama-3-70B TP=4 and TP=8: d_model 8192 (the fused all-reduce + RMSNorm row width), 64 query heads
  over 8 KV heads (TP=8: ONE KV head and 8 query heads per rank), FFN 28672 (a 3584-wide shard per
  rank at TP=8, 7168 at TP=4), a vocab-parallel LM head -- one layer, a small vocab (the shapes of a
  layer are what sharding can get wrong; 80 identical layers only take longer).
* Mixtral EP=8: 8 experts, one whole expert per rank, attention TP=8 (one KV head per rank).

Each compares greedy tokens and a sampled request's vocab-gathered logits with the TP=1 engine.
(BASELINE configs 3 and 5; SURVEY.md §2H. The reference has no parallelism at all.)"""
import dataclasses
import os
import queue
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp

from nats_llm_studio_amd.gguf.synth import SPECS, write_synthetic_gguf

L70 = dataclasses.replace(SPECS["llama-3-70b"], name="tp-70b-1layer", n_layer=1, vocab=4096, ctx=512)
MIX = dataclasses.replace(SPECS["mixtral-8x7b"], name="ep-mixtral-1layer", n_layer=1, d_ff=1024, vocab=4096,
                          ctx=512)
PROMPTS = [[1, 5, 9, 200, 31, 7, 77, 1000, 2048, 3], [1, 300, 301, 302]]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine(path, shard=None, comm=None):
    from nats_llm_studio_amd.engine.engine import Engine
    from nats_llm_studio_amd.gguf.reader import GGUFReader
    from nats_llm_studio_amd.models.llama import LlamaModel, ShardSpec
    m = LlamaModel(GGUFReader(path), "cpu", shard or ShardSpec(), comm)
    return Engine(m, None, max_batch=4, max_prefill_tokens=64, num_blocks=32, use_graphs=False, ctx=256)


def _run(eng):
    from nats_llm_studio_amd.engine.engine import GenRequest
    from nats_llm_studio_amd.engine.sampling import SamplingParams
    greedy = SamplingParams(max_tokens=4, ignore_eos=True)
    futs = [eng.submit(GenRequest(list(p), greedy)) for p in PROMPTS]
    while not all(f.done() for f in futs):
        eng.step()
    toks = [f.result().token_ids for f in futs]
    samp = SamplingParams(max_tokens=3, temperature=0.8, top_p=0.9, top_k=50, seed=5, ignore_eos=True)
    f = eng.submit(GenRequest(list(PROMPTS[0]), samp))
    while not f.done():
        eng.step()
    stoks = f.result().token_ids
    # the prefill logits of a one-token sampled request (TP: the vocab-parallel logits all-gather)
    one = SamplingParams(max_tokens=1, temperature=0.7, seed=3, ignore_eos=True)
    f = eng.submit(GenRequest(list(PROMPTS[1]), one))
    while not f.done():
        eng.step()
    lg = eng.full_logits if eng.full_logits is not None else eng.pb.logits
    return toks, stoks, lg[:1].clone()


def _worker(rank, world, port, path, ep, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from nats_llm_studio_amd.models import llama
    from nats_llm_studio_amd.models.llama import ShardSpec
    from nats_llm_studio_amd.parallel.comm import init_distributed
    import torch.distributed as dist
    if ep == "a2a":     # every step dispatches / combines over all-to-all (slices of 2 / 1 / 0 tokens per rank)
        llama._EP_A2A, llama._EP_A2A_T = "1", 1
    elif ep:
        llama._EP_A2A = "0"
    comm = init_distributed("cpu")
    try:
        eng = _engine(path, ShardSpec(rank, world, bool(ep)), comm)
        m = eng.model
        shapes = dict(Hq=m.Hq, Hkv=m.Hkv, ffn=m.ffn, experts=list(m.experts), vocab=m.vocab_hi - m.vocab_lo)
        if rank == 0:
            toks, stoks, lg = _run(eng)
            eng.stop_followers()
            out.put((rank, toks, stoks, lg.numpy(), dict(comm.stats), shapes))
        else:
            eng.follow()
            out.put((rank, None, None, None, None, shapes))
    finally:
        dist.destroy_process_group()


def _tp(path, world, ep=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, path, ep, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    t0 = time.time()
    try:
        while len(res) < world:
            try:
                r = q.get(timeout=2)
                res[r[0]] = r[1:]
            except queue.Empty:
                if any(p.exitcode not in (None, 0) for p in procs) or time.time() - t0 > 600:
                    raise AssertionError(f"TP workers failed: {[p.exitcode for p in procs]}")
    finally:
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    return res


@pytest.fixture(scope="module")
def l70(tmp_path_factory):
    path = str(tmp_path_factory.mktemp("tp70") / "tp-70b-1layer.gguf")
    write_synthetic_gguf(path, L70.name, "Q4_K_M", seed=3, spec=L70)
    return path, _run(_engine(path))


def _check(res, ref, vocab):
    ref_toks, ref_stoks, ref_lg = ref
    toks, stoks, lg, stats, _ = res[0]
    assert toks == ref_toks
    assert stoks == ref_stoks              # seeded: same u = uniform01(seed, position) on every path
    assert lg.shape[1] == vocab
    ref = ref_lg[:, :lg.shape[1]].numpy()
    err = abs(lg - ref).max() / (abs(ref).max() + 1e-6)
    assert err < 1e-3, err
    return stats


@pytest.mark.parametrize("world", [4, 8])
def test_llama70b_shapes_tp(l70, world):
    path, ref = l70
    res = _tp(path, world)
    stats = _check(res, ref, L70.vocab)
    for r in range(world):
        sh = res[r][4]
        assert sh["Hq"] == 64 // world and sh["Hkv"] == 8 // world and sh["ffn"] == 28672 // world, sh
    assert res[0][4]["ffn"] == (3584 if world == 8 else 7168)
    # per decode step and layer: O and down row-parallel sums of [rows, 8192] fp32, plus the vocab argmax
    assert stats["all_reduce"] > 0 and stats["all_reduce_bytes"] >= 2 * 8192 * 4


@pytest.mark.parametrize("mode", ["allreduce", "a2a"])
def test_mixtral_shapes_ep8(tmp_path, mode):
    """EP=8 both ways: combine-then-all-reduce, and dispatch / combine over all-to-all (LlamaModel._moe_a2a)."""
    path = str(tmp_path / "ep-mixtral-1layer.gguf")
    write_synthetic_gguf(path, MIX.name, "Q4_K_M", seed=4, spec=MIX)
    ref = _run(_engine(path))
    res = _tp(path, 8, ep="a2a" if mode == "a2a" else True)
    stats = _check(res, ref, MIX.vocab)
    assert (stats.get("all_to_all", 0) > 0) == (mode == "a2a"), stats
    assert [res[r][4]["experts"] for r in range(8)] == [[r] for r in range(8)]
    assert all(res[r][4]["Hkv"] == 1 for r in range(8))
