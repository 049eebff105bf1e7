"""Batch-1 decode experiment: a chain of N dependent M=1 GEMVs (x_{i+1} = f16(W_i x_i), 4096 x 4096 Q4_K, path A)
captured as one hipGraph, (a) serially on one stream, (b) overlapped: link i on stream i % 2 with no graph edge
to link i-1 -- each launch issues its weight prologue, then waits on the device for its producer's workgroups
(GemvArgs::dep). Per-link time and the bit-equality of the two chains' outputs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np
import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.gguf import quants as Q
from nats_llm_studio_amd.gguf.constants import GGMLType


def main(N=24, D=4096, waves=4, rt=1, reps=20):
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    ws = [ops.QWeight(Q.random_blocks(GGMLType.Q4_K, D * D, 0.02, rng), GGMLType.Q4_K, D, D, dev) for _ in range(N)]
    xs = [torch.zeros(16, D, dtype=ops.ACT_DTYPE, device=dev) for _ in range(N + 1)]
    xs[0][0] = (torch.randn(D, device=dev) * 0.5).to(ops.ACT_DTYPE)
    kw = dict(mode=0, waves=waves, rt=rt, ks=1)
    nwg = ops.gemv_grid([ops.Seg(ws[0])], rt)
    done = torch.zeros(N, dtype=torch.int32, device=dev)
    pas = torch.zeros(N, dtype=torch.int32, device=dev)

    def serial():
        for i in range(N):
            ops.qgemv([ops.Seg(ws[i])], xs[i], xs[i + 1], 1, epi="act", **kw)

    st = [torch.cuda.Stream(dev) for _ in range(2)]

    def overlapped():
        cur = torch.cuda.current_stream()
        for s in st:
            s.wait_stream(cur)
        for i in range(N):
            with torch.cuda.stream(st[i % 2]):
                ops.qgemv([ops.Seg(ws[i])], xs[i], xs[i + 1], 1, epi="act",
                          dep=(done[i - 1:i], nwg, pas[i:i + 1]) if i else None,
                          done=done[i:i + 1] if i + 1 < N else None, **kw)
        for s in st:
            cur.wait_stream(s)

    def branches_nodep():
        # the same two-stream graph without the device dependency (links race: timing only)
        cur = torch.cuda.current_stream()
        for s in st:
            s.wait_stream(cur)
        for i in range(N):
            with torch.cuda.stream(st[i % 2]):
                ops.qgemv([ops.Seg(ws[i])], xs[i], xs[i + 1], 1, epi="act", **kw)
        for s in st:
            cur.wait_stream(s)

    def serial_dep():
        # one stream, every link with the dependency machinery (its cost without any overlap)
        for i in range(N):
            ops.qgemv([ops.Seg(ws[i])], xs[i], xs[i + 1], 1, epi="act",
                      dep=(done[i - 1:i], nwg, pas[i:i + 1]) if i else None,
                      done=done[i:i + 1] if i + 1 < N else None, **kw)

    out = {}
    for name, fn in (("serial", serial), ("serial_dep", serial_dep), ("branches_nodep", branches_nodep),
                     ("overlapped", overlapped)):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3 / N)
        out[name] = (sorted(ts)[reps // 2], xs[N][0].clone())
        print(f"{name}: {out[name][0]:.2f} us per link (median of {reps} replays of {N} links)", flush=True)
    same = torch.equal(out["serial"][1], out["overlapped"][1]) and torch.equal(out["serial"][1], out["serial_dep"][1])
    print(f"outputs bit-equal: {same}; counters after: done {done.tolist()[:4]} pass {pas.tolist()[:4]}", flush=True)
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main(*[int(v) for v in sys.argv[1:]]))
