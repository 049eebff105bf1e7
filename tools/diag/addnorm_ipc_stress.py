"""W processes on ONE GPU run the tensor-parallel prefill pattern of the fused add+norm (csrc/kernels/allreduce.hip):
per call a row-parallel "GEMM" (a torch f16 matmul of the 70B o-projection shard) into the partial, then the one-shot
add+norm over IPC. Row counts cycle through the rehearsal's sizes. After every call each rank synchronises and reads
the error word; on the first error every rank prints its debug state and the device-clock history of the failed item
(t_start / t_pushed / t_polled on the 100 MHz wall clock that all processes share), then all stop.

    python tools/diag/addnorm_ipc_stress.py --world 4 --iters 40 [--rows 44,8,1,22]
"""
import argparse
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, a, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        from nats_llm_studio_amd.ops import _lib
        from nats_llm_studio_amd.parallel.comm import Comm
        from nats_llm_studio_amd.parallel.oneshot import OneShotAllReduce
        comm = Comm(dist.group.WORLD, dist.group.WORLD, dev)
        ar = OneShotAllReduce(comm)
        D, K = a.D, a.K
        g = torch.Generator(device="cpu").manual_seed(1234 + rank)
        w = (torch.randn(D, K, generator=g) * 0.02).half().to(dev)
        rows_seq = [int(v) for v in a.rows.split(",")]
        maxr = max(rows_seq)
        xin = (torch.randn(maxr, K, generator=g)).half().to(dev)
        x = torch.zeros(maxr, D, device=dev)
        part = torch.zeros(maxr, D, device=dev)
        h = torch.zeros(maxr, D, dtype=torch.float16, device=dev)
        nw = torch.ones(D, device=dev)
        L = _lib.lib()
        import numpy as np
        rng = np.random.default_rng(rank)
        t_launch = []
        bad = None
        for it in range(a.iters):
            T = rows_seq[it % len(rows_seq)]
            for _ in range(a.gemms):
                part[:T].copy_(torch.matmul(xin[:T], w.t()).float())
            if a.jitter:
                time.sleep(float(rng.random()) * a.jitter / 1e3)
            t_launch.append(time.time())
            ar.add_norm(part, x, nw, h, T, 1e-5)
            if a.batch > 1 and (it + 1) % a.batch:
                continue                   # async: the next call queues behind this one, no host sync
            torch.cuda.synchronize()
            e = int(ar.err.item())
            host = torch.zeros(32, dtype=torch.int32)
            _lib.check(L.nls_ar_err_words(ar.nbuf, ar.cap, ar.world, host.data_ptr(), 32,
                                          torch.cuda.current_stream().cuda_stream), "nls_ar_err_words")
            torch.cuda.synchronize()
            fl = torch.tensor([max(e, int(host[0]))], dtype=torch.int32)
            dist.all_reduce(fl, op=dist.ReduceOp.MAX)
            if int(fl):
                bad = it
                break
        out = dict(calls=len(t_launch), bad_call=bad)
        if bad is not None:
            st = ar.debug_state()
            out["state"] = {k: v for k, v in st.items() if not k.startswith("addnorm8192_epochs")}
            # the device-clock history of every item this rank or a peer reported as timed out
            items = set()
            w_ = st.get("timeout_addnorm", [0] * 8)
            if w_[0] and w_[6]:
                items.add((w_[1], w_[2]))
            objs = [None] * world
            dist.all_gather_object(objs, sorted(items))
            allitems = sorted({tuple(i) for lst in objs for i in lst})
            nblk = L.nls_ar_row_blocks(D)
            out["hist"] = {f"{b},{c}": ar._probe_hist(b * nblk + c) for b, c in allitems}
            out["t_launch_last"] = t_launch[-3:]
        dist.barrier()
        q.put((rank, out))
        ar.close()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        q.put((rank, {"exception": repr(e), "tb": traceback.format_exc()[-1500:]}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--rows", default="44,8,1,22,44,44,8")
    ap.add_argument("--D", type=int, default=8192)
    ap.add_argument("--K", type=int, default=2048)
    ap.add_argument("--gemms", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1, help="calls queued per host sync (async ranks)")
    ap.add_argument("--jitter", type=float, default=0.0, help="random host delay before each call, ms")
    a = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, a.world, port, a, q)) for r in range(a.world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(a.world):
            r, out = q.get(timeout=300)
            res[r] = out
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in sorted(res):
        print(f"rank {r}: {res[r]}", flush=True)
    return 0 if all(v.get("bad_call") is None and "exception" not in v for v in res.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
