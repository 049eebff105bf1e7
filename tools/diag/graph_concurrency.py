"""Do independent branches of a captured hipGraph run concurrently on MI355X? Two simulated one-shot ranks' fused
add+norm launches (SimulatedGroup.add_norm_rank: each waits for the other's push) are put on two forked streams --
eagerly, then captured as two parallel graph branches. Serial execution shows up as a timed-out poll (error word),
concurrency as clean sums. (Decides whether a decode graph could overlap a kernel with its predecessor.)"""
import sys

import torch

from nats_llm_studio_amd.parallel.oneshot import SimulatedGroup


def run(capture: bool, spins: int = 1 << 20):
    dev = torch.device("cuda:0")
    g = SimulatedGroup(2, 1 << 20, dev, max_spins=spins)
    D, rows = 4096, 2
    nw = torch.ones(D, device=dev)
    parts = [torch.randn(rows, D, device=dev) for _ in range(2)]
    xs = [torch.zeros(rows, D, device=dev) for _ in range(2)]
    hs = [torch.zeros(rows, D, dtype=torch.float16, device=dev) for _ in range(2)]
    s = [torch.cuda.Stream(dev) for _ in range(2)]

    def body():
        cur = torch.cuda.current_stream()
        for r in range(2):
            s[r].wait_stream(cur)
            with torch.cuda.stream(s[r]):
                g.add_norm_rank(r, parts[r], xs[r], nw, hs[r], rows, 1e-5, spins)
        for r in range(2):
            cur.wait_stream(s[r])
    if capture:
        gr = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(gr):
            body()
        for x in xs:
            x.zero_()
        g.err.zero_()
        torch.cuda.synchronize()
        gr.replay()
    else:
        body()
    torch.cuda.synchronize()
    ok = all(torch.allclose(x, parts[0] + parts[1], atol=1e-4) for x in xs)
    err = int(g.err.item())
    g.close()
    return ok, err


if __name__ == "__main__":
    for cap in (False, True):
        ok, err = run(cap)
        print(f"{'graph' if cap else 'eager'}: sums ok {ok}, timeout error word {err}", flush=True)
    sys.exit(0)
