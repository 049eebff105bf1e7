#!/usr/bin/env python3
"""The fused add+norm one-shot in SimulatedGroup (all ranks in one launch on one GPU) over calls of varying
row counts: per call, the rows whose normalised output h (or residual x) is off the fp32 reference, and the
error words. Launch options come from the environment (NLS_AR_RETAG / NLS_AR_POLL_INV, allreduce.hip ar_opts).
    python tools/addnorm_sim_probe.py [--world 2 --rows 16 --D 4096]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from nats_llm_studio_amd import ops
from nats_llm_studio_amd.parallel.oneshot import SimulatedGroup


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--rows", type=int, default=16)
    ap.add_argument("--D", type=int, default=4096)
    a = ap.parse_args()
    gpu = torch.device("cuda:0")
    torch.manual_seed(0)
    g = SimulatedGroup(a.world, 1 << 20, gpu)
    nw = (1 + 0.1 * torch.randn(a.D, device=gpu)).float()
    for it, rr in enumerate([a.rows, max(1, a.rows // 2), a.rows, a.rows, a.rows // 2, a.rows]):
        base = torch.randn(rr, a.D, device=gpu)
        parts = torch.randn(a.world, rr, a.D, device=gpu)
        xs = base.unsqueeze(0).repeat(a.world, 1, 1).contiguous()
        hs = torch.zeros(a.world, rr, a.D, dtype=ops.ACT_DTYPE, device=gpu)
        g.add_norm(parts, xs, nw, hs, rr, 1e-5)
        torch.cuda.synchronize()
        ref = base + parts.sum(0)
        href = ref * torch.rsqrt(ref.pow(2).mean(1, keepdim=True) + 1e-5) * nw
        bad_h = {r: [int(b) for b in ((hs[r].float() - href).abs().amax(1) > 0.05 * href.abs().amax()).nonzero().flatten()]
                 for r in range(a.world)}
        bad_x = {r: [int(b) for b in ((xs[r] - ref).abs().amax(1) > 1e-3).nonzero().flatten()] for r in range(a.world)}
        zero_h = {r: [int(b) for b in (hs[r].float().abs().amax(1) == 0).nonzero().flatten()] for r in range(a.world)}
        print(json.dumps(dict(call=it, rows=rr, err=int(g.err.item()), bad_h=bad_h, zero_h=zero_h, bad_x=bad_x,
                              env={k: os.environ.get(k) for k in ("NLS_AR_RETAG", "NLS_AR_POLL_INV")})), flush=True)
    g.close()


if __name__ == "__main__":
    main()
