"""Tensor/expert-parallel communicator.

The reference has no collectives at all (its only communication is NATS
request-reply, `/root/reference/nats_llm_studio.go:207-217`); multi-GPU execution was LM
Studio's concern. Here one process drives one GPU and the ranks of a model shard talk over
`torch.distributed` (backend "nccl" = RCCL over xGMI on MI355X, gloo on CPU for tests):

  * data plane (`group`): the row-parallel all-reduce after O-proj / down-proj (fused with
    the residual: rank 0's GEMV adds into the residual, the other ranks overwrite it with
    their partial, then ONE in-place sum), the MoE expert all-reduce, the vocab-parallel
    greedy argmax (an int64 MAX all-reduce of packed (value, index) keys -- 8 bytes per
    row instead of gathering [B, V] logits), and a logits all-gather only when a request
    samples. Small all-reduces can be routed to the IPC one-shot kernel
    (`parallel/oneshot.py`) instead of RCCL.
  * control plane: rank 0 (the scheduler) broadcasts each step's header + packed int32 metadata
    so follower ranks launch the same step -- through a shared-memory ring when the group is on
    one host (`parallel/shm_ctrl.py`), else over the gloo `ctrl` group.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from .. import ops
from ..ops import Seg

_SIGN = -(1 << 63)


class Comm:
    def __init__(self, group=None, ctrl_group=None, device=None):
        self.group = group
        self.ctrl = ctrl_group if ctrl_group is not None else group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        self.src = dist.get_global_rank(group, 0) if group is not None else 0
        self.device = torch.device(device) if device is not None else None
        self.oneshot = None          # optional small-message all-reduce (parallel/oneshot.py)
        # Eager calls (prefill chunks, capture warm-ups, first-use steps) take the IPC one-shot kernels too when
        # the message fits `cap` (round 5). Rounds 3-4 routed them to RCCL after eager add+norm calls timed out on
        # one MI355X shared by two ranks; the cause was scheduling, not visibility: one workgroup per (row, slice)
        # put ~1,700 polling waves on the GPU for a 52-row prefill chunk, the PEER rank's preceding GEMM could not
        # be scheduled, and its push came only after the bounded poll had expired (device-clock timestamps of both
        # ranks, profiles/tp_oneshot_eager_r05.txt). The fused add+norm now runs on a bounded grid (allreduce.hip).
        # NLS_ONESHOT_EAGER=0 sends eager calls to RCCL again.
        self.oneshot_eager = os.environ.get("NLS_ONESHOT_EAGER", "1") == "1"
        self.stats = dict(all_reduce=0, all_reduce_bytes=0, ctrl=0, ctrl_s=0.0)
        self.ring = None             # shared-memory control ring (ranks on one host), else gloo broadcasts
        if self.size > 1 and os.environ.get("NLS_SHM_CTRL", "1") == "1":
            import socket
            hosts = [None] * self.size
            dist.all_gather_object(hosts, socket.gethostname(), group=self.ctrl)
            if len(set(hosts)) == 1:
                from .shm_ctrl import ShmCtrlRing
                self.ring = ShmCtrlRing(self.ctrl, self.rank, self.size)

    # ------------------------------------------------------------------ data plane
    def _os(self, t: torch.Tensor):
        """The one-shot engine for a call on `t`, or None (RCCL)."""
        if self.oneshot is None or not t.is_cuda:
            return None
        if not self.oneshot_eager and not torch.cuda.is_current_stream_capturing():
            return None
        return self.oneshot

    def all_reduce(self, t: torch.Tensor, op=dist.ReduceOp.SUM):
        self.stats["all_reduce"] += 1
        self.stats["all_reduce_bytes"] += t.numel() * t.element_size()
        if op == dist.ReduceOp.SUM and self._os(t) is not None and self.oneshot.eligible(t):
            self.oneshot.all_reduce(t)
            self.stats["oneshot_all_reduce"] = self.stats.get("oneshot_all_reduce", 0) + 1
            return t
        dist.all_reduce(t, op=op, group=self.group)
        return t

    OVERLAP_ROWS = 256      # prefill: row chunk of the GEMM / all-reduce pipeline

    def row_parallel_add(self, w, xin: torch.Tensor, resid: torch.Tensor, T: int, alpha: float):
        """resid[:T] += alpha * sum_r x_r @ W_r^T  (W row-parallel: K split across ranks).
        Prefill-size T on GPUs: the GEMM runs in row chunks and chunk c's all-reduce runs on a side
        stream while chunk c+1's GEMM computes (RCCL overlapped with the dequant GEMM); the caller's
        stream waits for the last reduction."""
        epi = "add" if self.rank == 0 else "f32"
        C = self.OVERLAP_ROWS
        if not resid.is_cuda or T < 2 * C:
            ops.qgemv([Seg(w)], xin, resid, T, alpha=alpha, epi=epi)
            self.all_reduce(resid[:T])
            return
        cur = torch.cuda.current_stream(resid.device)
        if getattr(self, "_comm_stream", None) is None:
            self._comm_stream = torch.cuda.Stream(resid.device)
        cs = self._comm_stream
        for r0 in range(0, T, C):
            n = min(C, T - r0)
            ops.qgemv([Seg(w)], xin[r0:], resid[r0:], n, alpha=alpha, epi=epi)
            cs.wait_stream(cur)
            with torch.cuda.stream(cs):
                self.all_reduce(resid[r0:r0 + n])
        cur.wait_stream(cs)

    def row_parallel_add_norm(self, w, xin: torch.Tensor, part: torch.Tensor, resid: torch.Tensor,
                              nw: torch.Tensor, h: torch.Tensor, T: int, alpha: float, eps: float) -> bool:
        """Decode fast path: partial GEMV into `part`, then ONE fused one-shot kernel sums the ranks'
        partials in rank order into the residual and writes the next RMSNorm (h) -- 2 launches per
        row-parallel projection instead of GEMV + all-reduce + norm. False: not applicable (caller
        falls back to row_parallel_add + rmsnorm)."""
        os_ = self._os(resid)
        if os_ is None or not os_.addnorm_ok(T, resid.shape[1]):
            return False
        ops.qgemv([Seg(w)], xin, part, T, alpha=alpha, epi="f32")
        self.stats["all_reduce"] += 1
        self.stats["all_reduce_bytes"] += T * resid.shape[1] * 4
        os_.add_norm(part, resid, nw, h, T, eps)
        return True

    def vocab_parallel_argmax(self, keys: torch.Tensor, n: int, vocab_lo: int, next_ids: torch.Tensor):
        """Per-rank fused-argmax keys (value<<32 | ~local_idx) -> global greedy ids on every rank. Both paths
        leave keys[:n] re-armed (the next step's fused arg-max needs no reset launch)."""
        if self._os(keys) is not None:
            # one IPC launch: rebase, exchange, max, unpack and re-arm (no RCCL call in the decode graph)
            self.stats["all_reduce"] += 1
            self.stats["all_reduce_bytes"] += 8 * n
            self.oneshot.argmax(keys, n, vocab_lo, next_ids)
            return
        k = keys[:n]
        if keys.is_cuda:                       # device keys are unsigned: make signed order match
            k.bitwise_xor_(_SIGN)
        k.sub_(vocab_lo)                       # ~local_idx - lo == ~(local_idx + lo): global index
        self.all_reduce(k, op=dist.ReduceOp.MAX)
        if keys.is_cuda:
            k.bitwise_xor_(_SIGN)
        ops.argmax_unpack(keys, n, next_ids, rearm=True)

    def gather_logits(self, logits: torch.Tensor, n: int, vocab: int, per: int) -> torch.Tensor:
        """Vocab-sharded logits [n, Vs] -> full [n, vocab] on every rank (only when sampling)."""
        loc = torch.zeros(n, per, dtype=logits.dtype, device=logits.device)
        vs = min(per, logits.shape[1])
        loc[:, :vs] = logits[:n, :vs]
        out = torch.empty(self.size * n, per, dtype=logits.dtype, device=logits.device)
        dist.all_gather_into_tensor(out, loc, group=self.group)
        return out.view(self.size, n, per).permute(1, 0, 2).reshape(n, self.size * per)[:, :vocab]

    def gather_candidates(self, vals: torch.Tensor, idx: torch.Tensor):
        """Per-rank top-C candidates [n, C] (values, global ids; ops.topc_candidates) -> [n, size * C] on
        every rank, in rank order = vocabulary order (ranks hold consecutive vocab shards). 8 bytes per
        candidate instead of 4 per vocabulary entry: C = 128 at TP=8 moves 8 KiB per sampled row, not 500 KiB."""
        n, C = vals.shape
        os_ = self._os(vals)
        if os_ is not None and os_.gather_ok(2 * n * C):
            # lossless IPC all-gather of (values | ids) in one launch, rows already in vocabulary order
            self.stats["all_reduce"] += 1
            self.stats["all_reduce_bytes"] += 8 * n * C * self.size
            src = getattr(vals, "_packed", None)       # ops.topc_candidates' [2, n, C] block: gathered as it is
            if src is None or getattr(idx, "_packed", None) is not src:
                src = torch.stack([vals.contiguous().view(torch.int32), idx.contiguous().view(torch.int32)])
            dst = torch.empty(2, n, self.size * C, dtype=torch.int32, device=vals.device)
            os_.gather(src, dst)
            return dst[0].view(torch.float32), dst[1]
        ov = torch.empty(self.size * n, C, dtype=vals.dtype, device=vals.device)
        oi = torch.empty(self.size * n, C, dtype=idx.dtype, device=idx.device)
        dist.all_gather_into_tensor(ov, vals.contiguous(), group=self.group)
        dist.all_gather_into_tensor(oi, idx.contiguous(), group=self.group)
        self.stats["all_reduce"] += 1
        self.stats["all_reduce_bytes"] += 8 * n * C * self.size
        return (ov.view(self.size, n, C).permute(1, 0, 2).reshape(n, self.size * C),
                oi.view(self.size, n, C).permute(1, 0, 2).reshape(n, self.size * C))

    # ------------------------------------------------------------------ expert-parallel dispatch / combine
    def _staged(self, t: torch.Tensor) -> bool:
        """gloo moves host tensors only for all-to-all (the 1-GPU rehearsal's data group): stage through host."""
        return t.is_cuda and dist.get_backend(self.group) == "gloo"

    def exchange_counts(self, send: list) -> list:
        """send[r] = rows this rank sends to rank r -> recv[r] = rows rank r sends here (one int64 all-to-all)."""
        dev = self.device if (self.device is not None and self.device.type == "cuda"
                              and dist.get_backend(self.group) != "gloo") else torch.device("cpu")
        c = torch.tensor(send, dtype=torch.int64, device=dev)
        o = torch.empty_like(c)
        dist.all_to_all_single(o, c, group=self.group)
        return o.tolist()

    def all_to_all_rows(self, t: torch.Tensor, send: list, recv: list) -> torch.Tensor:
        """Rows of `t` grouped by destination (send[r] rows for rank r, in rank order) -> the rows every rank
        sent here, grouped by source rank (recv[r] rows from rank r). RCCL all-to-all over xGMI: each pair of
        ranks exchanges only its own rows on its own link."""
        staged = self._staged(t)
        src = (t.cpu() if staged else t).contiguous()
        out = src.new_empty((sum(recv),) + tuple(t.shape[1:]))
        dist.all_to_all_single(out, src, recv, send, group=self.group)
        self.stats["all_to_all"] = self.stats.get("all_to_all", 0) + 1
        self.stats["all_to_all_bytes"] = self.stats.get("all_to_all_bytes", 0) + src.numel() * src.element_size()
        return out.to(t.device) if staged else out

    def all_gather_rows(self, rows: torch.Tensor) -> torch.Tensor:
        """Equal-size row blocks [n, ...] of every rank -> [size * n, ...] in rank order."""
        staged = self._staged(rows)
        src = (rows.cpu() if staged else rows).contiguous()
        out = src.new_empty((self.size * src.shape[0],) + tuple(src.shape[1:]))
        dist.all_gather_into_tensor(out, src, group=self.group)
        self.stats["all_gather"] = self.stats.get("all_gather", 0) + 1
        return out.to(rows.device) if staged else out

    # ------------------------------------------------------------------ control plane
    def bcast_ctrl(self, t: torch.Tensor):
        """Host int32 tensor from rank 0 to all ranks: the shared-memory ring when every rank of the
        group is on this host (one memcpy + a sequence store per step), else a gloo broadcast."""
        import time
        self.stats["ctrl"] += 1
        t0 = time.perf_counter()
        if self.ring is not None:
            self.ring.bcast(t)
        else:
            dist.broadcast(t, src=self.src, group=self.ctrl)
        self.stats["ctrl_s"] += time.perf_counter() - t0
        return t

    def min_int(self, v: int) -> int:
        t = torch.tensor([int(v)], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.ctrl)
        return int(t.item())

    def barrier(self):
        dist.barrier(group=self.ctrl)


def init_distributed(device_type: Optional[str] = None, timeout_s: float = 600.0) -> Comm:
    """One process per GPU: reads RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT."""
    import datetime
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    local = int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device(f"cuda:{local}") if device_type == "cuda" else torch.device("cpu")
    if device_type == "cuda":
        torch.cuda.set_device(dev)
    if not dist.is_initialized():
        kw = dict(backend="nccl" if device_type == "cuda" else "gloo",
                  timeout=datetime.timedelta(seconds=timeout_s))
        if device_type == "cuda":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    ctrl = dist.new_group(backend="gloo") if device_type == "cuda" else None
    comm = Comm(dist.group.WORLD, ctrl, dev)
    if device_type == "cuda" and comm.size > 1 and os.environ.get("NLS_ONESHOT_AR", "1") == "1":
        from .oneshot import try_oneshot
        comm.oneshot = try_oneshot(comm)
    return comm
