"""Host side of the one-shot IPC all-reduce (`csrc/kernels/allreduce.hip`).

Each rank allocates one uncached receive buffer, exports it with hipIpcGetMemHandle, the
handles are exchanged over the (gloo) control group, and every rank maps its peers' buffers.
Decode-size fp32 sums (row-parallel O / down projections, MoE expert outputs) then cost one
kernel that pushes the message over all xGMI links at once -- no RCCL ring, capturable in
the decode hipGraph. Messages above `cap` floats fall back to RCCL (Comm.all_reduce).

On by default for TP on GPUs (NLS_ONESHOT_AR=0 disables; an IPC setup failure falls back to RCCL).
Row-parallel decode projections use the FUSED variant (`add_norm`): the ranks' partial sums, the
residual add and the next RMSNorm in one launch, each row spread over D/256 workgroups. A poll that
times out raises the error word of every rank; the engine fetches its word with each decode step's
tokens (`err_fetch`) and fails the step instead of returning wrong sums. `SimulatedGroup` runs the
same kernels for W "ranks" inside one process on one GPU -- the protocol test used on single-GPU
boxes, where cross-device IPC cannot be exercised.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import _lib

# floats per message (2 parity slots x world per buffer set): a 256-row prefill chunk of d = 8192 (Llama-3-70B) fits,
# so every tensor-parallel all-reduce of the engine runs on the IPC kernels (8 MiB; 384 MiB of buffers at TP=8)
DEFAULT_CAP = 256 * 8192
AG_MAX_WORDS = 16 * 64 * 256 * 2       # the gather kernel's fixed grid: AG_BLOCKS x AR_MAX_WG_BLOCKS x AG_THREADS granules


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
        # a third set for the lossless all-gather + fused vocab-parallel arg-max (ids, keys, sampling
        # candidates), again with epochs of its own
        self.gbuf, self.gpeers = self._exchange(L, hs, comm)
        if comm.min_int(int(self.ok)) == 0:
            self.close()
            raise RuntimeError("one-shot all-reduce: IPC buffer setup failed on some rank")
        dev = comm.device
        self.device = dev
        # ranks sharing this GPU (the one-GPU rehearsal): their polling grids shrink so that a peer's whole-CU
        # kernel still finds whole CUs (allreduce.hip nls_ar_set_norm_wgs); one rank per GPU keeps the full grids
        self.co_resident = _co_resident(comm, dev)
        if self.co_resident > 1:
            _lib.check(L.nls_ar_set_norm_wgs(max(8, (128 // (self.co_resident - 1)) & ~7)), "nls_ar_set_norm_wgs")
        # one epoch counter per slot block of the receive buffers (allreduce.hip SlotBlocks)
        self.epochs = torch.zeros(L.nls_ar_epoch_slots(self.cap), dtype=torch.int32, device=dev)
        self.gepochs = torch.zeros(L.nls_ag_epoch_slots(self.cap), dtype=torch.int32, device=dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self._norm = {}               # D -> (epochs, tickets, ssq) of the fused add+norm
        self.resets = 0
        self._trace = None
        if os.environ.get("NLS_TP_TRACE", "0") == "1":
            import collections
            self._trace = collections.deque(maxlen=64)
        self.ebuf = None              # expert-parallel decode exchange (ep_setup)
        self.ERR_WORDS = 3
        comm.barrier()

    def ep_setup(self, rows: int, D: int):
        """Receive buffers of the expert-parallel decode exchange (csrc/kernels/ep_exchange.hip) for up to `rows`
        (token, slot) rows of D floats; collective (every rank calls it, in the same order as the others)."""
        L = _lib.lib()
        need = L.nls_epx_bytes(rows, D)
        ar_cap = -(-(need - 256) // (8 * self.world)) + 4
        ar_cap += (-ar_cap) % 4
        bufs_before = len(self._owned)
        buf, peers = self._exchange(L, L.nls_ar_handle_size(), self.comm, cap=ar_cap)
        if self.comm.min_int(int(self.ok and len(self._owned) > bufs_before)) == 0:
            raise RuntimeError("expert-parallel exchange: IPC buffer setup failed on some rank")
        self.ebuf, self.epeers, self.e_rows, self.e_D = buf, peers, int(rows), int(D)
        self.egen = torch.zeros(L.nls_epx_wgs(), dtype=torch.int32, device=self.device)
        if self.co_resident > 1:
            _lib.check(L.nls_epx_set_wgs(max(8, L.nls_epx_wgs() // (self.co_resident - 1))), "nls_epx_set_wgs")
        st = torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(L.nls_epx_init(buf, self.e_rows, self.e_D, st), "nls_epx_init")
        torch.cuda.synchronize(self.device)
        self.ERR_WORDS = 4
        self.comm.barrier()

    def ep_ok(self, n: int, D: int) -> bool:
        return self.ebuf is not None and n <= self.e_rows and D == self.e_D

    def ep_exchange(self, y: torch.Tensor, n: int, sel: torch.Tensor, per: int):
        """y[:n] (f32, [n, D]): rows whose expert (sel[j], global id) belongs to this rank (sel // per == rank)
        are pushed to every peer; the other rows are filled with the peers' -- every rank ends with all n rows."""
        rc = _lib.lib().nls_epx_run(y.data_ptr(), y.stride(0), n, y.shape[1], sel.data_ptr(), per, self.rank,
                                    self.world, self.epeers, self.e_rows, self.egen.data_ptr(), self.err.data_ptr(),
                                    self.max_spins, int(os.environ.get("NLS_EPX_CHECK", "0") == "1"), _stream(y))
        _lib.check(rc, "nls_epx_run")

    def _exchange(self, L, hs, comm, cap: Optional[int] = None):
        buf = ctypes.c_void_p()
        handle = (ctypes.c_char * hs)()
        mine = b""
        if self.ok and L.nls_ar_alloc(self.cap if cap is None else cap, self.world, ctypes.byref(buf), handle) == 0:
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

    def _norm_state(self, D: int):
        st = self._norm.get(D)
        if st is None:
            st = _norm_buffers(self.cap, D, self.device)
            self._norm[D] = st
        return st

    def addnorm_ok(self, rows: int, D: int) -> bool:
        return D % 4 == 0 and rows * D <= self.cap

    def add_norm(self, part: torch.Tensor, x: torch.Tensor, nw: torch.Tensor, h: torch.Tensor, rows: int,
                 eps: float):
        """x[:rows] += sum over ranks of part[:rows] (rank order), h = f16(rmsnorm(x) * nw): one launch."""
        D = x.shape[1]
        ep, tk, sq = self._norm_state(D)
        if self._trace is not None:       # NLS_TP_TRACE: host launch times of the last 64 calls (debug_state)
            import time
            self._trace.append((round(time.time(), 4), int(rows), torch.cuda.is_current_stream_capturing()))
        rc = _lib.lib().nls_ar_addnorm(part.data_ptr(), part.stride(0), x.data_ptr(), x.stride(0), nw.data_ptr(),
                                       h.data_ptr(), h.stride(0), rows, D, float(eps), self.npeers, self.world,
                                       self.rank, self.cap, ep.data_ptr(), tk.data_ptr(), sq.data_ptr(),
                                       self.err.data_ptr(), self.max_spins, _stream(x))
        _lib.check(rc, "nls_ar_addnorm")
        return h

    def eligible(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() <= self.cap
                and t.numel() % 4 == 0)

    ERR_WORDS = 3      # one error word per buffer set (sum, fused add+norm, gather / arg-max[, EP exchange: 4])

    def err_fetch(self, host: torch.Tensor):
        """Enqueue the copy of this rank's error words (raised by ANY rank's timed-out poll, one per buffer
        set) into pinned int32 host[0:3] on the current stream; read them after the stream has passed."""
        L = _lib.lib()
        st = torch.cuda.current_stream(self.device).cuda_stream
        for i, b in enumerate((self.buf, self.nbuf, self.gbuf)):
            _lib.check(L.nls_ar_err_fetch(b, self.cap, self.world, host.data_ptr() + 4 * i, st), "nls_ar_err_fetch")
        if self.ebuf is not None:
            _lib.check(L.nls_epx_err_fetch(self.ebuf, self.e_rows, self.e_D, host.data_ptr() + 12, st),
                       "nls_epx_err_fetch")

    def err_clear(self):
        L = _lib.lib()
        st = torch.cuda.current_stream(self.device).cuda_stream
        for b in (self.buf, self.nbuf, self.gbuf):
            _lib.check(L.nls_ar_err_clear(b, self.cap, self.world, st), "nls_ar_err_clear")
        if self.ebuf is not None:
            _lib.check(L.nls_epx_err_clear(self.ebuf, self.e_rows, self.e_D, st), "nls_epx_err_clear")
        self.err.zero_()

    def debug_state(self, rows: int = 48) -> dict:
        """Small host snapshot of the protocol state (NLS_TP_TRACE): per-workgroup epochs of the three
        buffer sets (fused add+norm: first slice of each of the first `rows` rows) and the row tickets --
        compared across ranks, a divergence names the collective whose call counts differ."""
        torch.cuda.synchronize(self.device)
        out = dict(ar=self.epochs[:8].tolist(), gather=self.gepochs[:16].tolist())
        if self._trace is not None:
            out["host_addnorm_launches"] = list(self._trace)
        for D, (ep, tk, _sq) in self._norm.items():
            nblk = ep.numel() // tk.numel()
            e = ep.view(-1, nblk)[:rows]
            out[f"addnorm{D}"] = e[:, 0].tolist()
            # rows whose slices disagree with slice 0 (a workgroup that missed a call)
            out[f"addnorm{D}_ragged"] = {int(r): e[r].tolist() for r in range(e.shape[0])
                                         if int((e[r] != e[r, 0]).sum())}
            out[f"tickets{D}"] = tk[:rows].tolist()
        L = _lib.lib()
        st = torch.cuda.current_stream(self.device).cuda_stream
        # per buffer set: [error, a, b, epoch, peer, first dword seen (tag = low 2 bits), marker, kernel]
        # (add+norm: a row, b slice; the others: a granule, b granules of the call)
        for name, buf in (("sum", self.buf), ("addnorm", self.nbuf), ("gather", self.gbuf)):
            host = torch.zeros(32, dtype=torch.int32)
            _lib.check(L.nls_ar_err_words(buf, self.cap, self.world, host.data_ptr(), 32, st), "nls_ar_err_words")
            torch.cuda.synchronize(self.device)
            w = host.tolist()
            out[f"timeout_{name}"] = w[:8]
            if name == "addnorm" and w[24]:
                # NLS_AR_PROBE: a push of THIS rank that memory did not hold right after the store completed
                out["push_readback_mismatch"] = dict(row=w[25], slice=w[26], epoch=w[27], peer=w[28],
                                                     written=hex(w[29] & 0xFFFFFFFF), read_back=hex(w[30] & 0xFFFFFFFF),
                                                     col=w[31])
            if name == "addnorm" and w[6] and w[19]:
                # words 8..18: the granule the last poll saw, the lane's column, its XCD, the epoch counter
                # re-read at the timeout and the granule read by an atomic RMW; plus the slot as memory holds
                # it NOW (both parities) and this rank's epoch row -- compare with the peer's own dump
                b, c, ep, peer, col = w[1], w[2], w[3], w[4], w[12]
                out["addnorm_timeout_detail"] = dict(
                    row=b, slice=c, epoch=ep, peer=peer, col=col, seen=[hex(v & 0xFFFFFFFF) for v in w[8:12]],
                    xcc=w[13], epoch_counter_at_timeout=w[14], rmw_seen=[hex(v & 0xFFFFFFFF) for v in w[15:19]])
                slots = {}
                D = next(iter(self._norm)) if self._norm else 0
                for par in (0, 1):
                    pk = torch.zeros(4, dtype=torch.int32)
                    off = (par * self.world + peer) * self.cap + b * D + col
                    _lib.check(L.nls_ar_peek(buf, off, 4, pk.data_ptr(), st), "nls_ar_peek")
                    torch.cuda.synchronize(self.device)
                    slots[par] = [hex(v & 0xFFFFFFFF) for v in pk.tolist()]
                out["addnorm_timeout_detail"]["slot_memory_now"] = slots
                if D:
                    out["probe_hist_self"] = self._probe_hist(b * L.nls_ar_row_blocks(D) + c)
        for D, (ep, tk, _sq) in self._norm.items():
            nblk = ep.numel() // tk.numel()
            out[f"addnorm{D}_epochs_rows0_23"] = ep.view(-1, nblk)[:24].tolist()
        # the PUSHING side's view: for a peer whose add+norm poll timed out waiting for THIS rank, read that
        # slot through this rank's IPC mapping of the peer's buffer (where this rank's kernel wrote) -- compare
        # with the peer's own "slot_memory_now"; and whether an imported range overlaps this process's own
        # allocations (a mapping shorter than the buffer would let later allocations land inside it)
        D = next(iter(self._norm)) if self._norm else 0
        for p in range(self.world):
            if p == self.rank or not self.npeers[p]:
                continue
            host = torch.zeros(20, dtype=torch.int32)
            _lib.check(L.nls_ar_err_words(self.npeers[p], self.cap, self.world, host.data_ptr(), 20, st),
                       "nls_ar_err_words")
            torch.cuda.synchronize(self.device)
            w = host.tolist()
            if w[6] and w[19] and w[4] == self.rank and D:
                view = {}
                for par in (0, 1):
                    pk = torch.zeros(4, dtype=torch.int32)
                    off = (par * self.world + self.rank) * self.cap + w[1] * D + w[12]
                    _lib.check(L.nls_ar_peek(self.npeers[p], off, 4, pk.data_ptr(), st), "nls_ar_peek")
                    torch.cuda.synchronize(self.device)
                    view[par] = [hex(v & 0xFFFFFFFF) for v in pk.tolist()]
                out[f"pusher_view_of_rank{p}"] = dict(row=w[1], col=w[12], epoch=w[3], slot_memory=view,
                                                      probe_hist_pusher=self._probe_hist(
                                                          w[1] * L.nls_ar_row_blocks(D) + w[2]))
        nbytes = L.nls_ar_buffer_bytes(self.cap, self.world)
        imported = [(n, int(ptr)) for n, arr in (("sum", self.peers), ("addnorm", self.npeers), ("gather", self.gpeers))
                    for r, ptr in enumerate(arr) if ptr and r != self.rank]
        try:
            segs = [(s["address"], s["total_size"]) for s in torch.cuda.memory_snapshot()]
        except Exception:
            segs = []
        out["imported_overlaps"] = [dict(buf=n, ptr=hex(ptr), seg=hex(a), seg_bytes=sz) for n, ptr in imported
                                    for a, sz in segs if a < ptr + nbytes and ptr < a + sz]
        out["imported_ptrs"] = [(n, hex(ptr)) for n, ptr in imported]
        out["own_ptrs"] = [hex(int(b)) for b in (self.buf, self.nbuf, self.gbuf)]
        return out

    @staticmethod
    def _probe_hist(eidx: int):
        """NLS_AR_PROBE: this process's last nls_ar_probe_depth() (32) add+norm launches of workgroup slot `eidx`, oldest first, as
        (epoch, xcc, failed, t_start, t_pushed, t_polled) -- times in the device-wide 100 MHz clock, which two
        ranks sharing one GPU read identically (compare a timed-out poll with the peer's push)."""
        import numpy as np
        depth = _lib.lib().nls_ar_probe_depth()
        host = np.zeros(depth * 8, dtype=np.uint32)
        if _lib.lib().nls_ar_probe_hist(int(eidx), host.ctypes.data) != 0:
            return None
        recs = []
        for i in range(depth):
            w = host[8 * i:8 * i + 8]
            if not w[0]:
                continue
            t = [int(w[2 + 2 * k]) | (int(w[3 + 2 * k]) << 32) for k in range(3)]
            recs.append((int(w[0]), int(w[1] & 0xFF), int(w[1] >> 8), *t))
        return sorted(recs)

    def reset(self):
        """After a timed-out poll: put every rank's receive slots, epochs and tickets back to the freshly
        allocated state. A late peer may still have written granules nobody consumed, and a later call of
        the same parity could take them for current data once the 2-bit tag wraps; re-initialising is the
        only safe continuation. Collective: every rank calls it (the engine's _OP_RESET), and the barriers
        on both sides make sure no rank has a kernel in flight while the buffers are rewritten."""
        L = _lib.lib()
        torch.cuda.synchronize(self.device)
        self.comm.barrier()
        st = torch.cuda.current_stream(self.device).cuda_stream
        for b in (self.buf, self.nbuf, self.gbuf):
            _lib.check(L.nls_ar_reinit(b, self.cap, self.world, st), "nls_ar_reinit")
        if self.ebuf is not None:
            _lib.check(L.nls_epx_init(self.ebuf, self.e_rows, self.e_D, st), "nls_epx_init")
            self.egen.zero_()
        for t in [self.epochs, self.gepochs, self.err] + [x for st_ in self._norm.values() for x in st_]:
            t.zero_()
        torch.cuda.synchronize(self.device)
        self.comm.barrier()
        self.resets += 1

    def argmax(self, keys: torch.Tensor, n: int, vocab_lo: int, next_ids: torch.Tensor):
        """Vocab-parallel greedy pick in one launch: this rank's fused arg-max keys of rows [0, n) (its vocab
        shard starts at vocab_lo) -> the global token ids in next_ids on every rank; keys re-armed (0)."""
        if 4 * n > self.cap:
            raise ValueError(f"one-shot arg-max: {n} rows exceed the buffer")
        rc = _lib.lib().nls_ag_argmax(keys.data_ptr(), n, int(vocab_lo), next_ids.data_ptr(), self.gpeers,
                                      self.world, self.rank, self.cap, self.gepochs.data_ptr(), self.err.data_ptr(),
                                      self.max_spins, _stream(keys))
        _lib.check(rc, "nls_ag_argmax")

    def gather_ok(self, words: int) -> bool:
        return 2 * words <= self.cap and words <= AG_MAX_WORDS

    def gather(self, src: torch.Tensor, dst: torch.Tensor):
        """Lossless all-gather: src [A, rows, C] of 32-bit words (this rank) -> dst [A, rows, world * C] with
        rank p's words at columns [p * C, (p + 1) * C) of every row (C even)."""
        A, rows, C = src.shape
        if (src.element_size() != 4 or dst.element_size() != 4 or not src.is_contiguous() or not dst.is_contiguous()
                or tuple(dst.shape) != (A, rows, self.world * C) or C % 2 or not self.gather_ok(src.numel())):
            raise ValueError("one-shot gather: bad operands")
        rc = _lib.lib().nls_ag_run(src.data_ptr(), src.numel() // 2, dst.data_ptr(), C, rows * C, self.gpeers,
                                   self.world, self.rank, self.cap, self.gepochs.data_ptr(), self.err.data_ptr(),
                                   self.max_spins, _stream(src))
        _lib.check(rc, "nls_ag_run")
        return dst

    def all_reduce(self, t: torch.Tensor):
        rc = _lib.lib().nls_ar_run(t.data_ptr(), t.numel(), self.peers, self.world, self.rank, self.cap,
                                   self.epochs.data_ptr(), self.err.data_ptr(), self.max_spins, _stream(t))
        _lib.check(rc, "nls_ar_run")
        return t

    def check(self):
        """Raise if any rank's call timed out waiting for a peer (call outside graph capture)."""
        host = torch.zeros(self.ERR_WORDS, dtype=torch.int32, pin_memory=True)
        self.err_fetch(host)
        torch.cuda.current_stream(self.device).synchronize()
        if int(self.err.item()) or int(host.max()):
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


def _co_resident(comm, device) -> int:
    """How many ranks of `comm` drive the same physical GPU as this one (host name + PCI bus id; 1 = its own GPU)."""
    import socket
    try:
        p = torch.cuda.get_device_properties(device)
        key = (socket.gethostname(), getattr(p, "pci_domain_id", None), getattr(p, "pci_bus_id", None),
               getattr(p, "pci_device_id", None),
               str(getattr(p, "uuid", "")))
    except Exception:
        key = (socket.gethostname(), str(device))
    keys = [None] * comm.size
    dist.all_gather_object(keys, key, group=comm.ctrl)
    return sum(1 for k in keys if k == key)


def _norm_buffers(cap: int, D: int, device, world_sim: int = 0):
    """Per-workgroup epochs, per-row tickets and per-workgroup sum-of-squares shares of the fused
    add+norm for rows of D columns (rows <= cap // D); world_sim > 0: one set per simulated rank."""
    nblk = _lib.lib().nls_ar_row_blocks(D)
    rowcap = max(1, cap // D)
    lead = (world_sim,) if world_sim else ()
    return (torch.zeros(*lead, rowcap * nblk, dtype=torch.int32, device=device),
            torch.zeros(*lead, rowcap, dtype=torch.int32, device=device),
            torch.zeros(*lead, rowcap * nblk, dtype=torch.float32, device=device))


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
        nb = L.nls_ar_epoch_slots(self.cap)
        self.epochs = [torch.zeros(nb, dtype=torch.int32, device=device) for _ in range(world)]
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        self.streams = [torch.cuda.Stream(device) for _ in range(world)]
        self.nbufs = []
        for _ in range(world):
            b = ctypes.c_void_p()
            _lib.check(L.nls_ar_alloc(cap, world, ctypes.byref(b), None), "nls_ar_alloc")
            self.nbufs.append(b.value)
        self.npeers = (ctypes.c_void_p * world)(*self.nbufs)
        self.device = device
        self._norm = {}

    def add_norm(self, parts: torch.Tensor, xs: torch.Tensor, nw: torch.Tensor, hs: torch.Tensor, rows: int,
                 eps: float):
        """parts / xs (f32) and hs (f16): [world, rows, D]; every rank runs in ONE launch (blockIdx.y = rank),
        so the ranks are co-scheduled however streams map onto hardware queues."""
        D = xs.shape[2]
        if D not in self._norm:
            self._norm[D] = _norm_buffers(self.cap, D, self.device, self.world)
        ep, tk, sq = self._norm[D]
        rc = _lib.lib().nls_ar_addnorm_sim(parts.data_ptr(), parts.stride(1), xs.data_ptr(), xs.stride(1),
                                           nw.data_ptr(), hs.data_ptr(), hs.stride(1), rows, D, float(eps),
                                           self.npeers, self.world, 0, self.cap, ep.data_ptr(), tk.data_ptr(),
                                           sq.data_ptr(), self.err.data_ptr(), self.max_spins,
                                           torch.cuda.current_stream().cuda_stream, self.world,
                                           parts.stride(0), xs.stride(0), hs.stride(0), ep.stride(0), tk.stride(0),
                                           sq.stride(0))
        _lib.check(rc, "nls_ar_addnorm_sim")

    def add_norm_rank(self, rank: int, part: torch.Tensor, x: torch.Tensor, nw: torch.Tensor, h: torch.Tensor,
                      rows: int, eps: float, max_spins: int):
        """ONE rank's fused add+norm alone (the production launch; the other ranks never arrive): the
        fault-injection path of the bounded spin."""
        D = x.shape[1]
        if D not in self._norm:
            self._norm[D] = _norm_buffers(self.cap, D, self.device, self.world)
        ep, tk, sq = self._norm[D]
        rc = _lib.lib().nls_ar_addnorm(part.data_ptr(), part.stride(0), x.data_ptr(), x.stride(0), nw.data_ptr(),
                                       h.data_ptr(), h.stride(0), rows, D, float(eps), self.npeers, self.world, rank,
                                       self.cap, ep[rank].data_ptr(), tk[rank].data_ptr(), sq[rank].data_ptr(),
                                       self.err.data_ptr(), int(max_spins), torch.cuda.current_stream().cuda_stream)
        _lib.check(rc, "nls_ar_addnorm")

    def err_words(self) -> List[int]:
        """Every simulated rank's error words (both buffer sets), synchronously."""
        L = _lib.lib()
        host = torch.zeros(2 * self.world, dtype=torch.int32, pin_memory=True)
        st = torch.cuda.current_stream().cuda_stream
        for r in range(self.world):
            L.nls_ar_err_fetch(self.bufs[r], self.cap, self.world, host.data_ptr() + 8 * r, st)
            L.nls_ar_err_fetch(self.nbufs[r], self.cap, self.world, host.data_ptr() + 8 * r + 4, st)
        torch.cuda.current_stream().synchronize()
        return host.tolist()

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
