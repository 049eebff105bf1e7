"""Tensor / expert-parallel rehearsal of the REAL engine on ONE GPU: W processes share cuda:0, the
control plane is gloo + the shared-memory ring, and the data plane is the IPC one-shot kernels only
(`parallel/oneshot.py`: fused all-reduce + RMSNorm, plain all-reduce, lossless gather, vocab-parallel
arg-max), so every captured decode hipGraph is RCCL-free. Greedy and seeded top-k requests are decoded
with hipGraphs (`Engine.capture_all` on every rank, chained asynchronous decode, in-graph sampling under
TP) and compared with the same model at TP=1.

Multi-GPU boxes are the driver's; this is how the multi-rank decode path (BASELINE configs 3 and 5:
`/root/reference/README.md:478-484` scale-out) executes on hardware here. Ranks on
one GPU are co-scheduled on separate hardware queues; xGMI visibility itself needs >= 2 GPUs.

    python -m nats_llm_studio_amd.parallel.rehearsal --model llama-3-70b-2layer --world 2 [--ep]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time
from typing import Dict, List, Optional

PROMPTS = [[1, 5, 9, 200, 31, 7, 77], [1, 300, 301, 302], [1, 17, 400, 23, 9, 9, 9, 12, 31], [1, 2]]


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _requests(new_tokens: int, greedy_only: bool = False):
    from ..engine.sampling import SamplingParams
    greedy = SamplingParams(max_tokens=new_tokens, ignore_eos=True)
    topk = SamplingParams(max_tokens=new_tokens, temperature=0.8, top_k=40, top_p=0.95, repeat_penalty=1.1,
                          seed=7, ignore_eos=True)
    # the reference's canonical payload (`/root/reference/README.md:196-204`: temperature only, plus a seed so TP=1
    # and TP=2 draw the same stream): the omitted fields take LM Studio's preset (engine/sampling.py), top_k 40
    # included, so these rows are sampled in-graph like the explicit top-k ones
    canon = SamplingParams.from_request({"temperature": 0.7, "seed": 11, "max_tokens": new_tokens,
                                         "ignore_eos": True})
    return [(p, greedy) for p in PROMPTS] + ([] if greedy_only else [(p, topk) for p in PROMPTS]
                                             + [(p, canon) for p in PROMPTS[:2]])


def _sync(dev):
    import torch
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _engine(path: str, dev, shard=None, comm=None, graphs: bool = True):
    from ..engine.engine import Engine
    from ..gguf.reader import GGUFReader
    from ..models.llama import LlamaModel, ShardSpec
    m = LlamaModel(GGUFReader(path), dev, shard or ShardSpec(), comm)
    graphs = graphs and dev.type == "cuda" and os.environ.get("NLS_REHEARSAL_GRAPHS", "1") == "1"
    # NLS_REHEARSAL_PREFILL: a larger prefill chunk (long-prompt case: row-parallel prefill all-reduces in 256-row
    # chunks on the comm side stream, comm.row_parallel_add)
    mp = int(os.environ.get("NLS_REHEARSAL_PREFILL", "256"))
    return Engine(m, None, max_batch=8, max_prefill_tokens=mp, num_blocks=max(256, 2 * mp // 16 + 64),
                  use_graphs=graphs, ctx=max(512, mp + 64))


def _kernel_profile(eng, futs, steps: int) -> Dict:
    """torch.profiler (roctracer) around `steps` greedy decode steps of THIS rank: every kernel of the captured
    TP decode graph by name, count and device time. (rocprofv3 intercepts every process's queues, and the
    two ranks sharing the GPU must run concurrently for the IPC kernels to meet: under it a rank's poll
    times out, which the engine then reports as a one-shot timeout -- so the trace is taken in-process.)"""
    import torch
    from torch.profiler import ProfilerActivity, profile
    n = 0
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(steps):
            if all(f.done() for f in futs):
                break
            eng.step()
            n += 1
        eng._drain()
        torch.cuda.synchronize()
    kern = {}
    for ev in prof.events():
        if getattr(ev, "device_type", None) is None or "CUDA" not in str(ev.device_type):
            continue
        name = ev.name
        k = kern.setdefault(name, [0, 0.0])
        k[0] += 1
        dt = getattr(ev, "device_time_total", None)
        k[1] += float(dt if dt is not None else getattr(ev, "cuda_time_total", 0.0))
    rows = sorted(([v[0] / max(1, n), round(v[1] / max(1, n), 1), k] for k, v in kern.items()), key=lambda r: -r[1])
    return dict(steps=n, per_step=[[round(c, 2), us, nm[:90]] for c, us, nm in rows],
                rccl_kernels=[nm for _, _, nm in rows if "nccl" in nm.lower() or "rccl" in nm.lower()])


def graph_dump_summary(d: str) -> Dict:
    """NLS_GRAPH_DUMP=<d>: per captured graph (engine._capture: one `.nodes` file of kernel-node names), its
    kernel count by name and the nodes naming RCCL / NCCL -- the evidence that TP decode graphs are RCCL-free."""
    import collections
    import glob
    out = {}
    for f in sorted(glob.glob(os.path.join(d, "*.nodes"))):
        names = collections.Counter(ln.strip()[:100] for ln in open(f, errors="replace")
                                    if ln.strip() and not ln.startswith("#"))
        out[os.path.basename(f)] = dict(nodes=sum(names.values()), kernels=dict(names.most_common()),
                                        rccl_nodes=sum(c for k, c in names.items()
                                                       if "nccl" in k.lower() or "rccl" in k.lower()),
                                        # PyTorch's own kernels (at::native): none belong in a decode graph
                                        torch_nodes=sum(c for k, c in names.items()
                                                        if "at6native" in k or "at::native" in k))
    return out


def _drive(eng, new_tokens: int, profile_steps: int = 0, greedy_only: bool = False) -> Dict:
    """Leader: greedy requests, then seeded top-k requests (all in flight together); greedy_only: the
    greedy ones alone (every step takes the vocab-parallel arg-max path instead of in-graph sampling)."""
    from ..engine.engine import GenRequest
    eng.capture_all()
    reqs = _requests(new_tokens, greedy_only)
    t0 = time.perf_counter()
    futs = [eng.submit(GenRequest(list(p), sp)) for p, sp in reqs]
    steps = 0
    while not all(f.done() for f in futs):
        eng.step()
        steps += 1
    _sync(eng.dev)
    wall = time.perf_counter() - t0
    out = dict(tokens=[f.result().token_ids for f in futs], steps=steps, wall_s=round(wall, 3),
               counters=dict(eng.counters), graphs=[list(k) for k in sorted(eng.graphs)])
    long_len = int(os.environ.get("NLS_REHEARSAL_LONG", "0"))
    if long_len:
        # one long greedy prompt prefilled in ONE chunk (NLS_REHEARSAL_PREFILL >= its length)
        from ..engine.sampling import SamplingParams
        f = eng.submit(GenRequest([1] + [(37 * i) % 5000 + 10 for i in range(long_len - 1)],
                                  SamplingParams(max_tokens=4, ignore_eos=True)))
        while not f.done():
            eng.step()
        _sync(eng.dev)
        out["long_tokens"] = f.result().token_ids
    if os.environ.get("NLS_REHEARSAL_WAVES", "0") == "1":
        # batch-size churn: a wave whose requests end at different lengths (the decode batch shrinks through
        # the graph buckets 8 -> 4 -> 2 -> 1), then a second wave joining (back up to 8): rows idle for many
        # steps come back through other captured graphs
        from ..engine.sampling import SamplingParams
        waves = []
        for w in range(2):
            fs = [eng.submit(GenRequest(list(p) + [w + 3], SamplingParams(max_tokens=2 + 3 * j, ignore_eos=True)))
                  for j, p in enumerate(PROMPTS + PROMPTS)]
            waves.append(fs)
            for _ in range(4 if w == 0 else 10 ** 6):
                if all(f.done() for f in fs):
                    break
                eng.step()
        while not all(f.done() for ws in waves for f in ws):
            eng.step()
        _sync(eng.dev)
        out["waves_tokens"] = [[f.result().token_ids for f in ws] for ws in waves]
    if profile_steps:
        # a marker window for kernel traces: greedy-only decode steps after a host sync
        if os.environ.get("NLS_REHEARSAL_BARRIER", "0") == "1":
            import torch.distributed as dist
            eng.sync(lambda: (_sync(eng.dev), dist.barrier()))    # every rank idle before the window
        futs = [eng.submit(GenRequest(list(p), sp)) for p, sp in reqs[:len(PROMPTS)]]
        while any(s.n_prefilled < s.n_target for s in eng.running) or eng.waiting:
            eng.step()
        eng._drain()
        _sync(eng.dev)
        t1 = time.perf_counter()
        for _ in range(profile_steps):
            if all(f.done() for f in futs):
                break
            eng.step()
        eng._drain()
        _sync(eng.dev)
        out["profile_window_ms_per_step"] = round((time.perf_counter() - t1) / profile_steps * 1e3, 3)
        if eng.dev.type == "cuda":
            out["kernel_profile"] = _kernel_profile(eng, futs, profile_steps)
        while not all(f.done() for f in futs):
            eng.step()
    return out


def _device(kind: str):
    import torch
    if kind == "cpu":
        torch.set_num_threads(2)
        return torch.device("cpu")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    return dev


def _ref_main(path: str, new_tokens: int, q, kind: str = "cuda", greedy_only: bool = False):
    try:
        dev = _device(kind)
        eng = _engine(path, dev)
        q.put(("ref", _drive(eng, new_tokens, greedy_only=greedy_only)))
    except Exception as e:           # report, never hang the parent
        import traceback
        q.put(("ref", {"exception": repr(e), "tb": traceback.format_exc()[-2000:]}))


def _rank_main(rank: int, world: int, port: int, path: str, ep: bool, new_tokens: int, profile_steps: int, q,
               kind: str = "cuda", greedy_only: bool = False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    try:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = _device(kind)
        from ..models.llama import ShardSpec
        from .comm import Comm
        comm = Comm(dist.group.WORLD, dist.group.WORLD, dev)
        if dev.type == "cuda":
            from .oneshot import OneShotAllReduce
            comm.oneshot = OneShotAllReduce(comm)
        eng = _engine(path, dev, ShardSpec(rank, world, ep), comm)
        if rank == 0:
            try:
                res = _drive(eng, new_tokens, profile_steps, greedy_only)
            finally:
                eng.stop_followers()          # also on failure: followers must not wait for a next step
            res["comm"] = dict(comm.stats)
            res["oneshot_resets"] = comm.oneshot.resets if comm.oneshot is not None else None
            res["ctrl_transport"] = "shm-ring" if comm.ring is not None else "gloo"
            if comm.oneshot is not None:
                from ..ops import _lib
                res["co_resident"] = comm.oneshot.co_resident
                res["addnorm_wgs"] = _lib.lib().nls_ar_get_norm_wgs()
        else:
            eng.sync_hook = lambda: (_sync(dev), dist.barrier())
            eng.follow()
            res = dict(counters=dict(eng.counters), graphs=[list(k) for k in sorted(eng.graphs)])
        if comm.oneshot is not None:
            comm.oneshot.check()
        dist.barrier()
        q.put((rank, res))
        if comm.oneshot is not None:
            comm.oneshot.close()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        q.put((rank, {"exception": repr(e), "tb": traceback.format_exc()[-2000:]}))


def _collect(procs, q, n: int, timeout: float) -> Dict:
    import queue
    res = {}
    t0 = time.time()
    t_fail = None
    try:
        while len(res) < n:
            try:
                k, v = q.get(timeout=2)
                res[k] = v
                if "exception" in v and t_fail is None:
                    t_fail = time.time()
            except queue.Empty:
                if t_fail is not None and time.time() - t_fail > 30:
                    break                    # a rank failed: give the others 30 s, then stop waiting
                if time.time() - t0 > timeout:
                    raise TimeoutError(f"rehearsal: {len(res)}/{n} results after {timeout} s")
                dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
                if dead:
                    raise RuntimeError(f"rehearsal worker died: exit codes {dead}")
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return res


def run(path: str, world: int = 2, ep: bool = False, new_tokens: int = 8, ref: bool = True,
        profile_steps: int = 0, timeout: float = 400.0, device: str = "cuda", greedy_only: bool = False) -> Dict:
    """TP=1 reference (one process) then the W-rank run (W processes), each on cuda:0 (device="cpu": the
    same flow on gloo, for CPU tests of the driver); returns both."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    out = {}
    if ref:
        q = ctx.Queue()
        p = ctx.Process(target=_ref_main, args=(path, new_tokens, q, device, greedy_only))
        p.start()
        out["ref"] = _collect([p], q, 1, timeout)["ref"]
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, path, ep, new_tokens, profile_steps, q, device,
                                                  greedy_only))
             for r in range(world)]
    for p in procs:
        p.start()
    res = _collect(procs, q, world, timeout)
    out["tp"] = res.get(0)
    out["followers"] = [res.get(r) for r in range(1, world)]
    if os.environ.get("NLS_GRAPH_DUMP"):
        out["graph_dump"] = graph_dump_summary(os.environ["NLS_GRAPH_DUMP"])
    return out


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-70b-2layer")
    ap.add_argument("--ftype", default=None)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--ep", action="store_true")
    ap.add_argument("--tokens", type=int, default=8)
    ap.add_argument("--no-ref", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--greedy-only", action="store_true")
    ap.add_argument("--no-graphs", action="store_true", help="eager decode on every rank (NLS_REHEARSAL_GRAPHS=0)")
    ap.add_argument("--dir", default=os.environ.get("NLS_BENCH_DIR", "/tmp/nls_bench"))
    a = ap.parse_args(argv)
    if a.no_graphs:
        os.environ["NLS_REHEARSAL_GRAPHS"] = "0"        # inherited by the spawned ranks
    from ..gguf.synth import write_synthetic_gguf
    ft = a.ftype or ("Q5_K_M" if "mixtral" in a.model else "Q4_K_M")
    path = os.path.join(a.dir, f"{a.model}-{ft}.gguf")
    if not os.path.exists(path):
        os.makedirs(a.dir, exist_ok=True)
        write_synthetic_gguf(path, a.model, ft, seed=3)
    r = run(path, a.world, a.ep, a.tokens, ref=not a.no_ref, profile_steps=a.profile_steps,
            greedy_only=a.greedy_only)
    print(json.dumps(r), flush=True)
    ok = all("exception" not in (v or {"exception": 1}) for v in [r.get("tp")] + r["followers"])
    if ok and "ref" in r:
        ok = r["ref"].get("tokens") == r["tp"].get("tokens")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
