"""Host side of the one-shot IPC all-reduce (`csrc/kernels/allreduce.hip`).

Each rank allocates one uncached receive buffer, exports it with hipIpcGetMemHandle, the
handles are exchanged over the (gloo) control group, and every rank maps its peers' buffers.
Decode-size fp32 sums (row-parallel O / down projections, MoE expert outputs) then cost one
kernel that pushes the message over all xGMI links at once -- no RCCL ring, capturable in
the decode hipGraph. Messages above `cap` floats fall back to RCCL (Comm.all_reduce).

Enabled with NLS_ONESHOT_AR=1 (TP on GPUs). `SimulatedGroup` runs the same kernel for W
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
    def __init__(self, comm, cap: int = DEFAULT_CAP, max_spins: int = 1 << 22):
        L = _lib.lib()
        self.comm = comm
        self.world, self.rank = comm.size, comm.rank
        self.cap = int(cap)
        self.max_spins = int(max_spins)
        hs = L.nls_ar_handle_size()
        buf = ctypes.c_void_p()
        handle = (ctypes.c_char * hs)()
        _lib.check(L.nls_ar_alloc(self.cap, self.world, ctypes.byref(buf), handle), "nls_ar_alloc")
        self.buf = buf.value
        handles: List[Optional[bytes]] = [None] * self.world
        dist.all_gather_object(handles, bytes(handle), group=comm.ctrl)
        ptrs = []
        self._opened = []
        for r, h in enumerate(handles):
            if r == self.rank:
                ptrs.append(self.buf)
                continue
            p = ctypes.c_void_p()
            hb = (ctypes.c_char * hs).from_buffer_copy(h)
            _lib.check(L.nls_ar_open(hb, ctypes.byref(p)), "nls_ar_open")
            ptrs.append(p.value)
            self._opened.append(p.value)
        self.peers = (ctypes.c_void_p * self.world)(*ptrs)
        dev = comm.device
        self.epochs = torch.zeros(L.nls_ar_blocks(), dtype=torch.int32, device=dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        comm.barrier()

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
        if self.buf:
            L.nls_ar_free(ctypes.c_void_p(self.buf))
            self.buf = None


class SimulatedGroup:
    """W one-shot all-reduce 'ranks' in ONE process on ONE GPU (one stream each)."""

    def __init__(self, world: int, cap: int, device, max_spins: int = 1 << 20):
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
        for b in self.bufs:
            L.nls_ar_free(ctypes.c_void_p(b))
        self.bufs = []
