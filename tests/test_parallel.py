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
    return toks, lg[:1].clone()


def _worker(rank, world, port, path, ep, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from nats_llm_studio_amd.models.llama import ShardSpec
    from nats_llm_studio_amd.parallel.comm import init_distributed
    import torch.distributed as dist
    comm = init_distributed("cpu")
    try:
        eng = _engine(path, ShardSpec(rank, world, ep), comm)
        if rank == 0:
            toks, lg = _run(eng)
            eng.stop_followers()
            out.put((toks, lg.numpy(), comm.stats["all_reduce"]))
        else:
            eng.follow()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fam,ep", [("llama", False), ("granite", False), ("mixtral", False), ("mixtral", True)])
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
                toks, lg, n_ar = q.get(timeout=2)
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
    assert toks == ref_toks
    ref = ref_lg[:, :lg.shape[1]].numpy()
    assert lg.shape[1] == spec.vocab
    err = abs(lg - ref).max() / (abs(ref).max() + 1e-6)
    assert err < 1e-3, err
