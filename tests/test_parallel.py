"""Tensor / expert parallel equivalence on CPU: world_size 2 over gloo (127.0.0.1) through
the same sharding + comm + engine code the GPU path uses (RCCL there), compared with TP=1.

SURVEY.md §4 "Distributed (no cluster)": TP/EP math runs on CPU gloo; the reference itself
has no parallelism at all (§2H)."""
import dataclasses
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from nats_llm_studio_amd.gguf.synth import SPECS, write_synthetic_gguf

# TP=2 needs per-rank widths that are multiples of the 256-element K-quant super-block
_TP_SPECS = {
    "llama": dataclasses.replace(SPECS["tiny-llama"], name="tp-llama", d_ff=1024),
    "mixtral": dataclasses.replace(SPECS["tiny-mixtral"], name="tp-mixtral"),
    "granite": dataclasses.replace(SPECS["tiny-granite"], name="tp-granite", d_ff=1024),
    "qwen2": dataclasses.replace(SPECS["tiny-qwen2"], name="tp-qwen2", d_ff=1024),
}
PROMPTS = [[1, 5, 9, 200, 31, 7, 77], [1, 300, 301, 302]]


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
    return Engine(m, None, max_batch=4, max_prefill_tokens=64, num_blocks=64, use_graphs=False, ctx=256)


def _run(eng):
    from nats_llm_studio_amd.engine.engine import GenRequest
    from nats_llm_studio_amd.engine.sampling import SamplingParams
    greedy = SamplingParams(max_tokens=6, ignore_eos=True)
    futs = [eng.submit(GenRequest(list(p), greedy)) for p in PROMPTS]
    while not all(f.done() for f in futs):
        eng.step()
    toks = [f.result().token_ids for f in futs]
    # a sampling request exercises the vocab-sharded logits all-gather
    samp = SamplingParams(max_tokens=1, temperature=0.7, seed=3, ignore_eos=True)
    f = eng.submit(GenRequest(list(PROMPTS[0]), samp))
    while not f.done():
        eng.step()
    lg = eng.full_logits if eng.full_logits is not None else eng.pb.logits
    lg = lg[:1].clone()
    # top-k sampling with penalties: under TP the rows are drawn from the gathered per-rank top-128 candidates
    # (Engine._sample_candidates), which must give exactly the full-vocabulary sampler's tokens
    topk = SamplingParams(max_tokens=8, temperature=0.9, top_k=20, top_p=0.9, repeat_penalty=1.3,
                          presence_penalty=0.2, seed=11, ignore_eos=True)
    futs = [eng.submit(GenRequest(list(p), topk)) for p in PROMPTS]
    while not all(f.done() for f in futs):
        eng.step()
    toks.append([f.result().token_ids for f in futs])
    # penalties that RAISE history logits (repeat_penalty < 1, negative presence): the candidates are not exact
    # there, so these rows must take the full-logits path -- and still match the full-vocabulary sampler
    boost = SamplingParams(max_tokens=5, temperature=0.8, top_k=10, repeat_penalty=0.7, presence_penalty=-0.5,
                           seed=5, ignore_eos=True)
    futs = [eng.submit(GenRequest(list(p), boost)) for p in PROMPTS]
    while not all(f.done() for f in futs):
        eng.step()
    toks.append([f.result().token_ids for f in futs])
    # mixed batch: a candidate-exact top-k row beside a row that forces the host-sampled path (repeat_penalty
    # < 1). While both run, every TP step samples on the host; once the short one finishes, the long row goes
    # back to the in-step sampler, whose penalty history ring must hold the tokens the host drew meanwhile.
    mix_long = SamplingParams(max_tokens=12, temperature=0.9, top_k=40, repeat_penalty=3.0, presence_penalty=1.0,
                              seed=21, ignore_eos=True)
    mix_short = SamplingParams(max_tokens=4, temperature=0.8, top_k=10, repeat_penalty=0.7, seed=22,
                               ignore_eos=True)
    futs = [eng.submit(GenRequest(list(PROMPTS[0]), mix_long)), eng.submit(GenRequest(list(PROMPTS[1]), mix_short))]
    while not all(f.done() for f in futs):
        eng.step()
    toks.append([f.result().token_ids for f in futs])
    return toks, lg


def _worker(rank, world, port, path, ep, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from nats_llm_studio_amd.models import llama
    from nats_llm_studio_amd.models.llama import ShardSpec
    if ep == "a2a":
        # every EP step (prefill of two prompts and decode) dispatches / combines over all-to-all
        llama._EP_A2A, llama._EP_A2A_T = "1", 1
    elif ep:
        llama._EP_A2A = "0"
    from nats_llm_studio_amd.parallel.comm import init_distributed
    import torch.distributed as dist
    comm = init_distributed("cpu")
    try:
        eng = _engine(path, ShardSpec(rank, world, bool(ep)), comm)
        if rank == 0:
            toks, lg = _run(eng)
            eng.stop_followers()
            out.put((toks, lg.numpy(), comm.stats["all_reduce"], dict(eng.counters, all_to_all=comm.stats.get("all_to_all", 0))))
        else:
            eng.follow()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fam,ep", [("llama", False), ("granite", False), ("mixtral", False), ("mixtral", True),
                                    ("mixtral", "a2a"), ("qwen2", False)])
def test_tp2_matches_tp1(tmp_path, fam, ep):
    spec = _TP_SPECS[fam]
    path = str(tmp_path / f"{spec.name}.gguf")
    write_synthetic_gguf(path, spec.name, "Q4_K_M", seed=1, spec=spec)
    ref_toks, ref_lg = _run(_engine(path))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, path, ep, q)) for r in range(2)]
    for p in procs:
        p.start()
    import queue
    import time
    t0 = time.time()
    try:
        while True:
            try:
                toks, lg, n_ar, ctr = q.get(timeout=2)
                break
            except queue.Empty:
                if any(p.exitcode not in (None, 0) for p in procs) or time.time() - t0 > 300:
                    raise AssertionError(f"TP workers failed: {[p.exitcode for p in procs]}")
    finally:
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    assert n_ar > 0
    assert (ctr["all_to_all"] > 0) == (ep == "a2a"), ctr
    # the top-k requests' decode steps drew from the gathered candidates INSIDE the step (in-graph sampler,
    # chained decode); only their first tokens (after prefill) were drawn on the host
    assert ctr["device_sampled_steps"] > 0, ctr
    assert ctr["candidate_sampled_prefills"] > 0 and ctr["candidate_sampled_steps"] == 0, ctr
    assert toks == ref_toks
    ref = ref_lg[:, :lg.shape[1]].numpy()
    assert lg.shape[1] == spec.vocab
    err = abs(lg - ref).max() / (abs(ref).max() + 1e-6)
    assert err < 1e-3, err


def _tp_worker_main(rank, world, port, argv):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from nats_llm_studio_amd import worker
    raise SystemExit(worker.main(argv))


def test_tp_worker_serves_chat_over_nats(tmp_path):
    """torchrun-style TP=2 worker: both ranks load shards, rank 0 answers lmstudio.chat_model
    over NATS, the follower executes every step; SIGTERM releases both."""
    import json
    import signal
    import time
    from nats_llm_studio_amd.natsio import Client, EmbeddedServer
    spec = _TP_SPECS["llama"]
    d = tmp_path / "models" / "synthetic" / "tp-llama-GGUF"
    d.mkdir(parents=True)
    write_synthetic_gguf(str(d / "tp-llama-Q4_K_M.gguf"), spec.name, "Q4_K_M", seed=2, spec=spec)
    srv = EmbeddedServer().start()
    argv = ["--nats-url", srv.url, "--models-dir", str(tmp_path / "models"), "--tp", "2", "--model", "tp-llama",
            "--max-batch", "4", "--max-ctx", "256", "--device", "cpu"]
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_tp_worker_main, args=(r, 2, port, argv)) for r in range(2)]
    for p in procs:
        p.start()
    cli = Client().connect(srv.url)
    try:
        deadline = time.time() + 120
        r = None
        while time.time() < deadline:
            try:
                r = json.loads(cli.request("lmstudio.health", b"{}", 2).data)
                break
            except Exception:
                assert all(p.exitcode in (None, 0) for p in procs), [p.exitcode for p in procs]
                time.sleep(0.5)
        assert r and r["ok"] and r["data"]["models_loaded"] == ["tp-llama"]
        body = {"model": "tp-llama", "messages": [{"role": "user", "content": "hello there"}], "max_tokens": 5,
                "temperature": 0}
        r = json.loads(cli.request("lmstudio.chat_model", json.dumps(body).encode(), 120).data)
        assert r["ok"] is True and r["data"]["http_status"] == 200, r
        assert r["data"]["response"]["usage"]["completion_tokens"] >= 1
        r2 = json.loads(cli.request("lmstudio.chat_model", json.dumps(body).encode(), 120).data)
        assert r2["data"]["response"]["choices"][0]["message"]["content"] == \
            r["data"]["response"]["choices"][0]["message"]["content"]
    finally:
        cli.close()
        os.kill(procs[0].pid, signal.SIGTERM)
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.kill()
        srv.stop()
    assert [p.exitcode for p in procs] == [0, 0]


def test_rehearsal_driver_cpu(tmp_path):
    """The one-GPU TP rehearsal driver (parallel/rehearsal.py) end to end on gloo: TP=1 reference process,
    then 2 ranks; greedy + seeded top-k tokens equal, sampled decode rows drawn by the in-step sampler."""
    from nats_llm_studio_amd.parallel import rehearsal
    spec = _TP_SPECS["llama"]
    path = str(tmp_path / "tp-llama.gguf")
    write_synthetic_gguf(path, spec.name, "Q4_K_M", seed=4, spec=spec)
    r = rehearsal.run(path, world=2, new_tokens=5, timeout=240, device="cpu")
    assert "exception" not in r["tp"], r["tp"]
    assert "exception" not in r["followers"][0], r["followers"][0]
    assert r["tp"]["tokens"] == r["ref"]["tokens"]
    c = r["tp"]["counters"]
    assert c["device_sampled_steps"] > 0 and c["candidate_sampled_steps"] == 0, c
    assert r["followers"][0]["counters"]["device_sampled_steps"] == c["device_sampled_steps"]
    # greedy-only batches: every step on the vocab-parallel arg-max, batch churn (waves of requests ending at
    # different lengths), plus the post-run marker window
    import os
    os.environ["NLS_REHEARSAL_WAVES"] = "1"
    try:
        g = rehearsal.run(path, world=2, new_tokens=5, timeout=240, device="cpu", greedy_only=True, profile_steps=3)
    finally:
        os.environ.pop("NLS_REHEARSAL_WAVES", None)
    assert "exception" not in g["tp"], g["tp"]
    assert g["tp"]["tokens"] == g["ref"]["tokens"] == r["ref"]["tokens"][:len(rehearsal.PROMPTS)]
    assert g["tp"]["waves_tokens"] == g["ref"]["waves_tokens"]
    assert g["tp"]["counters"]["device_sampled_steps"] == 0


def _a2a_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from nats_llm_studio_amd.parallel.comm import init_distributed
    import torch.distributed as dist
    comm = init_distributed("cpu")
    try:
        # rank r sends (r + d) % 3 rows to rank d (some zero), each row tagged (source, destination, index)
        send = [(rank + d) % 3 for d in range(world)]
        rows = torch.tensor([[rank, d, i] for d in range(world) for i in range(send[d])], dtype=torch.float32)
        recv = comm.exchange_counts(send)
        got = comm.all_to_all_rows(rows.view(-1, 3), send, recv)
        back = comm.all_to_all_rows(got, recv, send)           # the inverse exchange restores the original rows
        blk = torch.full((2, 4), float(rank))
        gathered = comm.all_gather_rows(blk)
        out.put((rank, recv, got.tolist(), bool(torch.equal(back, rows.view(-1, 3))), gathered.tolist()))
    finally:
        dist.destroy_process_group()


def test_comm_all_to_all_rows_uneven():
    """Comm.exchange_counts / all_to_all_rows / all_gather_rows (the EP dispatch / combine primitives) over
    gloo at world 3 with uneven and empty splits: rows arrive grouped by source rank in send order, and the
    inverse exchange restores every rank's rows."""
    import queue
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_a2a_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r = q.get(timeout=120)
            res[r[0]] = r[1:]
    except queue.Empty:
        raise AssertionError(f"workers failed: {[p.exitcode for p in procs]}")
    finally:
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.kill()
    for d in range(world):
        recv, got, inverse_ok, gathered = res[d]
        assert recv == [(s + d) % 3 for s in range(world)]
        assert got == [[s, d, i] for s in range(world) for i in range((s + d) % 3)]
        assert inverse_ok
        assert gathered == [[float(r)] * 4 for r in range(world) for _ in range(2)]
