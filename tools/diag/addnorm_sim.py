"""Diagnose the simulated-rank fused add+norm (SimulatedGroup.add_norm): per call, which rows of h disagree with
the fp32 reference, whether those rows look unwritten (zero), normalised with the pre-add x, or otherwise wrong,
and the row tickets left behind. Run with NLS_AR_RETAG=0/1 to compare."""
import sys

import torch

from nats_llm_studio_amd.parallel.oneshot import SimulatedGroup


def main(world=2, rows=16, D=4096, iters=8):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    g = SimulatedGroup(world, 1 << 20, dev)
    nw = (1 + 0.1 * torch.randn(D, device=dev)).float()
    bad_calls = 0
    for it in range(iters):
        rr = rows if it % 2 == 0 else max(1, rows // 2)
        base = torch.randn(rr, D, device=dev)
        parts = torch.randn(world, rr, D, device=dev)
        xs = base.unsqueeze(0).repeat(world, 1, 1).contiguous()
        hs = torch.zeros(world, rr, D, dtype=torch.float16, device=dev)
        g.add_norm(parts, xs, nw, hs, rr, 1e-5)
        torch.cuda.synchronize()
        ref = base + parts.sum(0)
        href = ref * torch.rsqrt(ref.pow(2).mean(1, keepdim=True) + 1e-5) * nw
        hpre = base * torch.rsqrt(ref.pow(2).mean(1, keepdim=True) + 1e-5) * nw
        x_ok = bool(torch.allclose(xs[0], ref, rtol=1e-5, atol=1e-5))
        rep = []
        for r in range(world):
            err = (hs[r].float() - href).abs().amax(1)
            for b in torch.nonzero(err > 0.02 * href.abs().amax()).flatten().tolist():
                row = hs[r, b].float()
                kind = ("zero" if row.abs().max() == 0 else
                        "pre-add" if (row - hpre[b]).abs().max() < 0.05 else "other")
                badc = torch.nonzero((row - href[b]).abs() > 0.02 * href.abs().amax()).flatten()
                rep.append(dict(rank=r, row=b, kind=kind, bad_cols=badc.numel(),
                                first_bad_slices=sorted({int(c) // 256 for c in badc[:64].tolist()})[:8]))
        _, tk, _ = g._norm[D]
        tks = tk[:, :rows].tolist()
        # NLS_AR_XCHECK=1: the normaliser's own re-sum of x^2 vs the slices' shares (words 32..38 of the error area)
        from nats_llm_studio_amd.ops import _lib
        xc = []
        for r in range(world):
            host = torch.zeros(8, dtype=torch.int32, pin_memory=True)
            _lib.lib().nls_ar_peek(g.nbufs[r], 2 * world * g.cap + 32, 8, host.data_ptr(),
                                   torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            w = host.tolist()
            if w[0] == 0xD44:
                import struct
                f = lambda u: struct.unpack("f", struct.pack("i", u))[0]
                xc.append(dict(rank=r, row=w[1], shares=round(f(w[2]), 3), reread=round(f(w[3]), 3), ep=w[4],
                               xcc=w[6]))
        print(f"call {it} rows {rr} x_ok {x_ok} err {int(g.err.item())} bad {rep[:6]} tickets_nonzero "
              f"{[[i for i, v in enumerate(t) if v] for t in tks]} xcheck {xc}", flush=True)
        bad_calls += bool(rep) or not x_ok
    g.close()
    return 1 if bad_calls else 0


if __name__ == "__main__":
    a = [int(v) for v in sys.argv[1:]]
    sys.exit(main(*a))
