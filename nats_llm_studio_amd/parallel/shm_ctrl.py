"""Host control plane for tensor-parallel replicas on ONE node: a shared-memory broadcast ring.

Rank 0 of a TP group schedules every step and the followers replay it (engine.Engine.follow), so
each decode step carries a small header + the packed int32 step metadata from rank 0 to every
other rank. Over gloo that is two TCP broadcasts per step; here it is a memcpy into a POSIX
shared-memory ring plus a sequence-number store, and followers poll it.

Ring layout (one SharedMemory segment, little-endian, x86 TSO):
  [0:8)                     writer sequence of the last published message
  [8:8+8*W)                 per-rank acknowledged sequence (followers write theirs)
  slot k at HDR + k*SLOT:   [seq:int64][nbytes:int64][payload ...]
A message is published by writing its payload, then its length, then its sequence number (stores
are not reordered with older stores on x86); a follower that sees slot.seq == expected reads a
complete payload. The writer reuses a slot only after every follower acknowledged the message that
last occupied it, so a slow follower never loses a step.
"""
from __future__ import annotations

import time
from multiprocessing import shared_memory
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

SLOTS = 8


class ShmCtrlRing:
    def __init__(self, group, rank: int, world: int, max_bytes: int = 1 << 20, name: Optional[str] = None):
        self.rank, self.world = rank, world
        self.slot_bytes = 16 + ((max_bytes + 63) // 64) * 64
        self.hdr = 64 + 8 * ((world + 7) // 8 * 8)
        size = self.hdr + SLOTS * self.slot_bytes
        if rank == 0:
            self.shm = shared_memory.SharedMemory(create=True, size=size)
            obj = [self.shm.name]
        else:
            obj = [None]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        if rank != 0:
            self.shm = shared_memory.SharedMemory(name=obj[0])
        buf = self.shm.buf
        self.mem = np.frombuffer(buf, dtype=np.uint8)
        self.acks = np.frombuffer(buf, dtype=np.int64, count=world, offset=8)
        self.seq = 0                                   # last sequence written (rank 0) / read (followers)
        if rank == 0:
            self.acks[:] = 0
            np.frombuffer(buf, dtype=np.int64, count=1, offset=0)[0] = 0
        dist.barrier(group=group)
        import atexit
        atexit.register(self.close)        # drop the numpy views before the segment is unmapped

    def _slot(self, seq: int):
        off = self.hdr + (seq % SLOTS) * self.slot_bytes
        head = np.frombuffer(self.shm.buf, dtype=np.int64, count=2, offset=off)
        return off, head

    @staticmethod
    def _wait(cond, timeout: float):
        t0 = time.perf_counter()
        spins = 0
        while not cond():
            spins += 1
            if spins > 2000:                        # ~ a few hundred us of spinning, then nap
                time.sleep(50e-6)
                if time.perf_counter() - t0 > timeout:
                    raise TimeoutError("shm control ring: peer did not respond")

    def bcast(self, t: torch.Tensor, timeout: float = 1800.0) -> torch.Tensor:
        """Same contract as dist.broadcast from rank 0 on a host tensor (receivers know the size)."""
        a = t.numpy() if t.is_contiguous() else t.contiguous().numpy()
        raw = a.view(np.uint8).reshape(-1)
        n = raw.size
        if n + 16 > self.slot_bytes:
            raise ValueError(f"control message of {n} bytes exceeds the ring slot")
        if self.rank == 0:
            seq = self.seq + 1
            if seq > SLOTS:                            # slot reuse: every follower acked seq - SLOTS
                need = seq - SLOTS
                self._wait(lambda: int(self.acks[1:].min()) >= need, timeout)
            off, head = self._slot(seq)
            self.mem[off + 16:off + 16 + n] = raw
            head[1] = n
            head[0] = seq                               # publish last
            np.frombuffer(self.shm.buf, dtype=np.int64, count=1, offset=0)[0] = seq
            self.seq = seq
        else:
            seq = self.seq + 1
            off, head = self._slot(seq)
            self._wait(lambda: int(head[0]) == seq, timeout)
            m = int(head[1])
            if m != n:
                raise RuntimeError(f"shm control ring: expected {n} bytes, got {m}")
            raw[:] = self.mem[off + 16:off + 16 + n]
            if not t.is_contiguous():
                t.copy_(torch.from_numpy(a))
            self.acks[self.rank] = seq
            self.seq = seq
        return t

    def close(self):
        if getattr(self, "shm", None) is None:
            return
        try:
            self.mem = self.acks = None
            import gc
            gc.collect()
            self.shm.close()
            if self.rank == 0:
                self.shm.unlink()
        except Exception:
            pass
        self.shm = None
