"""Host side of the one-shot IPC all-reduce (`csrc/kernels/allreduce.hip`).

Each rank allocates one uncached receive buffer, exports it with hipIpcGetMemHandle, the
handles are exchanged over the (gloo) control group, and every rank maps its peers' buffers.
Decode-size fp32 sums (row-parallel O / down projections, MoE expert outputs) then cost one
kernel that pushes the message over all xGMI links at once -- no RCCL ring, capturable in
the decode hipGraph. Messages above `cap` floats fall back to RCCL (Comm.all_reduce).

On by default for TP on GPUs (NLS_ONESHOT_AR=0 disables; an IPC setup failure falls back to RCCL).
Row-parallel decode projections use the FUSED variant (`add_norm`): the ranks' partial sums, the
residual add and the next RMSNorm in one launch. `SimulatedGroup` runs the same kernels for W
"ranks" inside one process on one GPU (one stream per rank) -- the protocol test used on
single-GPU boxes, where cross-device IPC cannot be exercised.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import _lib

DEFAULT_CAP = 64 * 4096 * 4          # floats: B=64 x d=16384 fp32 (8 MiB message), 2 slots x world


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


class OneShotAllReduce:
    def __init__(self, comm, cap: int = DEFAULT_CAP, max_spins: int = 1 << 24):
        L = _lib.lib()
        self.comm = comm
        self.world, self.rank = comm.size, comm.rank
        self.cap = int(cap)
        self.max_spins = int(max_spins)
        self._owned, self._opened = [], []
        hs = L.nls_ar_handle_size()
        # every rank runs every collective below whatever fails locally (a rank that raised early
        # would leave its peers blocked in all_gather); success is agreed on at the end
        self.ok = True
        self.buf, self.peers = self._exchange(L, hs, comm)
        # a second buffer set for the fused all-reduce + residual + RMSNorm (its own epoch counters:
        # the two protocols must never read each other's granules)
        self.nbuf, self.npeers = self._exchange(L, hs, comm)
        if comm.min_int(int(self.ok)) == 0:
            self.close()
            raise RuntimeError("one-shot all-reduce: IPC buffer setup failed on some rank")
        dev = comm.device
        self.epochs = torch.zeros(L.nls_ar_blocks(), dtype=torch.int32, device=dev)
        self.nepochs = torch.zeros(max(1, self.cap // 1024), dtype=torch.int32, device=dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        comm.barrier()

    def _exchange(self, L, hs, comm):
        buf = ctypes.c_void_p()
        handle = (ctypes.c_char * hs)()
        mine = b""
        if self.ok and L.nls_ar_alloc(self.cap, self.world, ctypes.byref(buf), handle) == 0:
            self._owned.append(buf.value)
            mine = bytes(handle)
        else:
            self.ok = False
        handles: List[Optional[bytes]] = [None] * self.world
        dist.all_gather_object(handles, mine, group=comm.ctrl)
        ptrs = []
        for r, h in enumerate(handles):
            if r == self.rank:
                ptrs.append(buf.value)
                continue
            p = ctypes.c_void_p()
            if self.ok and h and L.nls_ar_open((ctypes.c_char * hs).from_buffer_copy(h), ctypes.byref(p)) == 0:
                self._opened.append(p.value)
                ptrs.append(p.value)
            else:
                self.ok = False
                ptrs.append(None)
        return buf.value, (ctypes.c_void_p * self.world)(*ptrs)

    def addnorm_ok(self, rows: int, D: int) -> bool:
        return rows * D <= self.cap and rows <= self.nepochs.numel() and D <= 16 * 512

    def add_norm(self, part: torch.Tensor, x: torch.Tensor, nw: torch.Tensor, h: torch.Tensor, rows: int,
                 eps: float):
        """x[:rows] += sum over ranks of part[:rows] (rank order), h = f16(rmsnorm(x) * nw): one launch."""
        D = x.shape[1]
        rc = _lib.lib().nls_ar_addnorm(part.data_ptr(), part.stride(0), x.data_ptr(), x.stride(0), nw.data_ptr(),
                                       h.data_ptr(), h.stride(0), rows, D, float(eps), self.npeers, self.world,
                                       self.rank, self.cap, self.nepochs.data_ptr(), self.err.data_ptr(),
                                       self.max_spins, _stream(x))
        _lib.check(rc, "nls_ar_addnorm")
        return h

    def eligible(self, t: torch.Tensor) -> bool:
        return t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() <= self.cap

    def all_reduce(self, t: torch.Tensor):
        rc = _lib.lib().nls_ar_run(t.data_ptr(), t.numel(), self.peers, self.world, self.rank, self.cap,
                                   self.epochs.data_ptr(), self.err.data_ptr(), self.max_spins, _stream(t))
        _lib.check(rc, "nls_ar_run")
        return t

    def check(self):
        """Raise if any call timed out waiting for a peer (call outside graph capture)."""
        if int(self.err.item()):
            raise RuntimeError("one-shot all-reduce timed out waiting for a peer")

    def close(self):
        L = _lib.lib()
        for p in self._opened:
            L.nls_ar_close(ctypes.c_void_p(p))
        self._opened = []
        for b in self._owned:
            L.nls_ar_free(ctypes.c_void_p(b))
        self._owned = []
        self.buf = None


def try_oneshot(comm) -> Optional["OneShotAllReduce"]:
    """The IPC one-shot all-reduce for `comm`, or None (RCCL only) when the peer mapping fails."""
    try:
        return OneShotAllReduce(comm)
    except Exception as e:        # e.g. no IPC between these devices: RCCL still works
        print(f"[nls] one-shot all-reduce disabled ({e}); using RCCL", flush=True)
        return None


class SimulatedGroup:
    """W one-shot all-reduce 'ranks' in ONE process on ONE GPU (one stream each)."""

    def __init__(self, world: int, cap: int, device, max_spins: int = 1 << 24):
        L = _lib.lib()
        self.world, self.cap, self.max_spins = world, cap, max_spins
        self.bufs = []
        for _ in range(world):
            b = ctypes.c_void_p()
            _lib.check(L.nls_ar_alloc(cap, world, ctypes.byref(b), None), "nls_ar_alloc")
            self.bufs.append(b.value)
        self.peers = (ctypes.c_void_p * world)(*self.bufs)
        nb = L.nls_ar_blocks()
        self.epochs = [torch.zeros(nb, dtype=torch.int32, device=device) for _ in range(world)]
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        self.streams = [torch.cuda.Stream(device) for _ in range(world)]
        self.nbufs = []
        for _ in range(world):
            b = ctypes.c_void_p()
            _lib.check(L.nls_ar_alloc(cap, world, ctypes.byref(b), None), "nls_ar_alloc")
            self.nbufs.append(b.value)
        self.npeers = (ctypes.c_void_p * world)(*self.nbufs)
        self.nepochs_all = torch.zeros(world, max(1, cap // 1024), dtype=torch.int32, device=device)

    def add_norm(self, parts: torch.Tensor, xs: torch.Tensor, nw: torch.Tensor, hs: torch.Tensor, rows: int,
                 eps: float):
        """parts / xs (f32) and hs (f16): [world, rows, D]; every rank runs in ONE launch (blockIdx.y = rank),
        so the ranks are co-scheduled however streams map onto hardware queues."""
        D = xs.shape[2]
        ep = self.nepochs_all
        rc = _lib.lib().nls_ar_addnorm_sim(parts.data_ptr(), parts.stride(1), xs.data_ptr(), xs.stride(1),
                                           nw.data_ptr(), hs.data_ptr(), hs.stride(1), rows, D, float(eps),
                                           self.npeers, self.world, 0, self.cap, ep.data_ptr(), self.err.data_ptr(),
                                           self.max_spins, torch.cuda.current_stream().cuda_stream, self.world,
                                           parts.stride(0), xs.stride(0), hs.stride(0), ep.stride(0))
        _lib.check(rc, "nls_ar_addnorm_sim")

    def all_reduce(self, tensors: List[torch.Tensor]):
        L = _lib.lib()
        cur = torch.cuda.current_stream()
        for r, (t, s) in enumerate(zip(tensors, self.streams)):
            s.wait_stream(cur)
            rc = L.nls_ar_run(t.data_ptr(), t.numel(), self.peers, self.world, r, self.cap,
                              self.epochs[r].data_ptr(), self.err.data_ptr(), self.max_spins, s.cuda_stream)
            _lib.check(rc, "nls_ar_run")
        for s in self.streams:
            cur.wait_stream(s)

    def close(self):
        L = _lib.lib()
        for b in self.bufs + self.nbufs:
            L.nls_ar_free(ctypes.c_void_p(b))
        self.bufs = []
        self.nbufs = []
