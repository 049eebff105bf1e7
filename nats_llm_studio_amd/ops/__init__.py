"""Device ops. CUDA(HIP) tensors -> hand-written gfx950 kernels in `_kernels.so`;
CPU tensors -> the pure-torch fp32 reference of the same op (tests, CPU stub runs).

The CPU branch is never taken for GPU tensors: a missing kernel library on a GPU
box raises instead of silently running eager PyTorch.
"""
from __future__ import annotations

import ctypes
import math
import warnings
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..gguf.constants import GGMLType, GGML_BLOCK
from ..gguf.quants import dequantize
from . import _lib
from . import transcode

EPI = {"f32": 0, "act": 1, "add": 2, "swiglu": 3, "slabs": 4, "argmax": 5, "rope": 6}
import os as _os
# Path-A row-parallel GEMVs of up to this many rows run the next RMSNorm in their last workgroup.
# Off by default: measured on MI355X at batch 1 it LENGTHENS the step (2.43 vs 2.25 ms/token) -- the
# last workgroup's ticket + acquire + row reload sit on the critical path and cost more than the
# separate norm launch inside a hipGraph (profiles/rocprof_b1_r02_addnorm.txt). NLS_ADDNORM=8 enables.
ADDNORM_MAX_M = int(_os.environ.get("NLS_ADDNORM", "0"))
# Large-M GEMMs switch to the dense f16 kernel (mode 4, csrc/kernels/hgemm.hip) from this many rows
# on, for weights that carry an f16 copy (QWeight.expand_dense)
DENSE_MIN_M = int(_os.environ.get("NLS_DENSE_GEMM_M", "128"))
# launch config of the mapped-row (MoE expert) path-A GEMV: mode, waves, row tiles, split
# (Mixtral-8x7B batch 1 / 16, profiles/moe_selected_experts.txt: 0,4,2,1 3.90 / 10.0 ms per step vs 0,8,1,1
# 4.94 / 15.1)
MOE_GEMV = tuple(int(v) for v in _os.environ.get("NLS_MOE_GEMV", "0,4,2,1").split(","))
# Every large-M projection runs on the hand-written dense GEMMs (modes 4/5/10, tuning "d:" entries). The
# library GEMM that r02-r03 dispatched for some shapes ("mode 7": hipBLASLt via torch.mm + a separate epilogue)
# is gone from the engine; tools/dense_tune.py keeps measuring against it as the reference
# (profiles/dense_tune_r04.jsonl).
ACT_DTYPE = torch.float16   # activation dtype of every GEMM/GEMV input and SwiGLU/RMSNorm/attention output


def _stream_ptr(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


# ---------------------------------------------------------------------------
# Quantised weights
# ---------------------------------------------------------------------------

def to_device_layout(raw: np.ndarray, ggml_type: int, rows: int, K: int) -> np.ndarray:
    """ggml block bytes -> the "rows" layout (embedding tables; see csrc/kernels/common.h)."""
    t = GGMLType(ggml_type)
    raw = np.ascontiguousarray(raw).view(np.uint8).reshape(-1)
    if t == GGMLType.Q6_K:
        b = raw.reshape(-1, 210)
        return np.concatenate([b[:, 0:128].reshape(-1), b[:, 128:192].reshape(-1), b[:, 192:208].reshape(-1),
                               b[:, 208:210].reshape(-1)])
    if t == GGMLType.Q8_0:
        b = raw.reshape(-1, 34)
        return np.concatenate([b[:, 2:34].reshape(-1), b[:, 0:2].reshape(-1)])
    return raw


TILE_BYTES = {GGMLType.Q4_K: 2304, GGMLType.Q5_K: 2816, GGMLType.Q6_K: 3360, GGMLType.Q8_0: 4352,
              GGMLType.F16: 8192, GGMLType.BF16: 8192, GGMLType.F32: 16384}


def tile_layout(raw: torch.Tensor, ggml_type: int, rows: int, K: int) -> torch.Tensor:
    """ggml block bytes (uint8 tensor, any device) -> the GEMV "tiled" layout: rows padded to
    16, one contiguous tile-block per (16-row tile, 256-value super-block), arranged so every
    wave-wide 16-B load reads 1 KiB contiguous (csrc/kernels/common.h)."""
    t = GGMLType(ggml_type)
    nb = K // 256
    rp = (rows + 15) // 16 * 16
    T = rp // 16
    rb = row_bytes(t, K)
    b = raw.reshape(rows, rb)
    if rp != rows:
        b = torch.cat([b, torch.zeros(rp - rows, rb, dtype=torch.uint8, device=b.device)])
    if t in (GGMLType.Q4_K, GGMLType.Q5_K):
        bs = 144 if t == GGMLType.Q4_K else 176
        q0 = 16 if t == GGMLType.Q4_K else 48
        B = b.reshape(T, 16, nb, bs)
        parts = [B[..., 0:16].permute(0, 2, 1, 3).reshape(T, nb, 256)]
        if t == GGMLType.Q5_K:        # QH[g][r][8]: qh bytes 8g..8g+7
            parts.append(B[..., 16:48].reshape(T, 16, nb, 4, 8).permute(0, 2, 3, 1, 4).reshape(T, nb, 512))
        # P_h[g][r] = chunk 2h bytes 8g..+8 | chunk 2h+1 bytes 8g..+8   (qs byte = 32c + 8g + i)
        qs = B[..., q0:q0 + 128].reshape(T, 16, nb, 2, 2, 4, 8)
        parts.append(qs.permute(0, 2, 3, 5, 1, 4, 6).reshape(T, nb, 2048))
    elif t == GGMLType.Q6_K:
        B = b.reshape(T, 16, nb, 210)
        ql = B[..., 0:128].reshape(T, 16, nb, 2, 2, 4, 8)          # ql byte = 64n + 32run + 8g + i
        qh = B[..., 128:192].reshape(T, 16, nb, 2, 4, 8)           # qh byte = 32n + 8g + i
        parts = [ql.permute(0, 2, 3, 5, 1, 4, 6).reshape(T, nb, 2048),     # QL_n[g][r][run][8]
                 qh.permute(0, 2, 4, 1, 3, 5).reshape(T, nb, 1024),        # QH[g][r][n][8]
                 B[..., 192:208].permute(0, 2, 1, 3).reshape(T, nb, 256),
                 B[..., 208:210].permute(0, 2, 1, 3).reshape(T, nb, 32)]
    elif t == GGMLType.Q8_0:
        B = b.reshape(T, 16, nb, 8, 34)
        d = B[..., 0:2].permute(0, 2, 1, 3, 4).reshape(T, nb, 256)
        qs = B[..., 2:34].reshape(T, 16, nb, 4, 2, 4, 8)           # block 2p + bb, byte 8g + i
        parts = [qs.permute(0, 2, 3, 5, 1, 4, 6).reshape(T, nb, 4096), d]
    elif t in (GGMLType.F16, GGMLType.BF16):
        parts = [b.reshape(T, 16, nb, 8, 4, 16).permute(0, 2, 3, 4, 1, 5).reshape(T, nb, 8192)]
    elif t == GGMLType.F32:
        parts = [b.reshape(T, 16, nb, 8, 4, 2, 16).permute(0, 2, 3, 5, 4, 1, 6).reshape(T, nb, 16384)]
    else:
        raise NotImplementedError(f"tiled layout for {t.name}")
    out = torch.cat(parts, dim=2) if len(parts) > 1 else parts[0]
    assert out.shape[2] == TILE_BYTES[t]
    return out.reshape(-1).contiguous()


def row_bytes(ggml_type: int, K: int) -> int:
    blk, nb = GGML_BLOCK[GGMLType(ggml_type)]
    return K // blk * nb


class QWeight:
    """A [rows, K] weight matrix resident on `device` in its quantised form.

    layout="tiled" (GEMV/GEMM operands) or "rows" (embedding tables, row gathers). `gtype` is the GGUF
    block type of the file; `type` the format the kernels execute (the same, except for the formats
    ops/transcode.py re-encodes at load: Q4_0/Q4_1/Q5_0/Q5_1 -> Q51, Q3_K -> Q6_K, Q2_K -> F16)."""

    def __init__(self, raw: np.ndarray, ggml_type: int, rows: int, K: int, device, name: str = "",
                 layout: str = "tiled"):
        self.gtype = int(ggml_type)
        self.type = int(ggml_type)
        self.rows = int(rows)
        self.K = int(K)
        self.name = name
        self.layout = layout
        self.device = torch.device(device)
        if K % 256:
            raise ValueError(f"{name}: K={K} is not a multiple of 256")
        with warnings.catch_warnings():     # read-only mmap views: copied below
            warnings.simplefilter("ignore", UserWarning)
            if GGMLType(ggml_type) in transcode.TRANSCODED:
                t = torch.from_numpy(np.ascontiguousarray(np.asarray(raw).view(np.uint8).reshape(-1)))
                t = t.to(self.device) if self.device.type != "cpu" else t
                t, self.type = transcode.device_form(t, ggml_type, rows, K, layout)
                if layout == "rows":
                    t = torch.from_numpy(np.ascontiguousarray(to_device_layout(t.cpu().numpy(), self.type, rows, K)))
                    self.data = t.to(self.device) if self.device.type != "cpu" else t.clone()
                elif self.type == transcode.QT_Q51:
                    self.data = t
                else:
                    self.data = tile_layout(t, self.type, rows, K)
            elif layout == "rows":
                t = torch.from_numpy(np.ascontiguousarray(to_device_layout(raw, ggml_type, rows, K)))
                self.data = t.to(self.device) if self.device.type != "cpu" else t.clone()
            else:
                t = torch.from_numpy(np.ascontiguousarray(np.asarray(raw).view(np.uint8).reshape(-1)))
                t = t.to(self.device) if self.device.type != "cpu" else t
                self.data = tile_layout(t, ggml_type, rows, K)
        self._raw = np.ascontiguousarray(raw).view(np.uint8).reshape(-1) if self.device.type == "cpu" else None
        self._dense = None
        self.d16: Optional[torch.Tensor] = None    # row-major f16 copy for the large-M GEMM (mode 4)

    def to_f16(self) -> "QWeight":
        """This matrix re-encoded as tiled F16 (its dequantised values): for a fused launch whose segments
        would otherwise need two kernel type-sets (e.g. a Q2_K model's Q|K|V with a Q3_K V)."""
        if self.device.type == "cpu" or self.type == int(GGMLType.F16):
            return self
        w = QWeight.__new__(QWeight)
        w.__dict__.update(self.__dict__)
        w.type = int(GGMLType.F16)
        w.data = tile_layout(self.dense(torch.float16).contiguous().view(torch.uint8).reshape(-1), GGMLType.F16,
                             self.rows, self.K)
        w.d16 = None
        return w

    def expand_dense(self) -> int:
        """Keep a dequantised row-major f16 copy next to the quantised tiles (GPU; idempotent).
        Returns the bytes it added. Large-M GEMMs then run on MFMA without in-kernel dequantisation;
        the copy is the HIP dequant kernel's output, i.e. the very f16 values modes 2/3 feed their MFMAs."""
        if self.device.type != "cuda" or self.layout != "tiled" or self.d16 is not None:
            return 0
        self.d16 = self.dense(torch.float16).contiguous()
        return self.d16.numel() * 2

    @staticmethod
    def expand_dense_group(ws: Sequence["QWeight"]) -> int:
        """expand_dense for matrices launched together as adjacent output columns (a layer's Q|K|V): their f16
        copies become consecutive row ranges of ONE buffer, so a dense launch sees a single segment (_seg_arr
        merges them) -- no partial weight tile at each segment end, e.g. 64 whole 96-row tiles for Llama-3-8B's
        6144 Q|K|V rows instead of 43 + 11 + 11. Falls back to per-matrix copies when shapes or devices differ."""
        ws = list(ws)
        if (len(ws) < 2 or any(w.device.type != "cuda" or w.layout != "tiled" or w.d16 is not None for w in ws)
                or len({w.K for w in ws}) != 1 or len({str(w.device) for w in ws}) != 1):
            return sum(w.expand_dense() for w in ws)
        buf = torch.empty(sum(w.rows for w in ws), ws[0].K, dtype=torch.float16, device=ws[0].device)
        r0 = 0
        for w in ws:
            buf[r0:r0 + w.rows].copy_(w.dense(torch.float16))
            w.d16 = buf[r0:r0 + w.rows]
            r0 += w.rows
        return buf.numel() * 2

    @property
    def dense_bytes(self) -> int:
        return self.rows * self.K * 2

    @property
    def nbytes(self) -> int:
        return self.data.numel()

    def dense(self, dtype=torch.float32) -> torch.Tensor:
        """Dequantised [rows, K] (CPU: numpy ggml codec; GPU: HIP dequant kernel, f16)."""
        if self.device.type == "cpu":
            if self._dense is None:
                self._dense = torch.from_numpy(dequantize(self._raw, self.gtype, (self.rows, self.K)).copy())
            return self._dense.to(dtype)
        out = torch.empty(self.rows, self.K, dtype=ACT_DTYPE, device=self.device)
        _lib.check(_lib.lib().nls_dequant(self.data.data_ptr(), self.type, self.rows, self.K, out.data_ptr(),
                                          self.K, _stream_ptr(out)), "nls_dequant")
        return out.to(dtype)


def kernel_set(types) -> Optional[int]:
    """The HIP kernel type-set that runs one launch over segments of these device types, None if no single
    set covers them (csrc/kernels/qgemv.hip: Q6_K joins any quantised set, Q8_0 sets 1 and 3)."""
    ts = set(int(t) for t in types)
    flt = ts & {0, 1, 30}
    q4k, q5k, q8, q51 = 12 in ts, 13 in ts, 8 in ts, transcode.QT_Q51 in ts
    if ts - {0, 1, 30, 8, 12, 13, 14, transcode.QT_Q51}:
        return None
    if (flt and ts - flt) or (q4k and (q5k or q8 or q51)) or (q51 and q5k):
        return None
    return 2 if flt else (3 if q51 else (0 if q4k else (1 if (q5k or q8) else 0)))


def interleave_gate_up(gate_raw: np.ndarray, up_raw: np.ndarray, ggml_type: int, rows: int, K: int,
                       group: int = 8) -> np.ndarray:
    """Rows [g0..g7, u0..u7, g8..g15, u8..u15, ...] so one 16-row MFMA tile yields 8 SwiGLU outputs."""
    rb = row_bytes(ggml_type, K)
    g = np.asarray(gate_raw).view(np.uint8).reshape(rows // group, group, rb)
    u = np.asarray(up_raw).view(np.uint8).reshape(rows // group, group, rb)
    return np.ascontiguousarray(np.concatenate([g, u], axis=1)).reshape(-1)


@dataclass
class Seg:
    w: QWeight
    ycol: int = 0
    xmap: Optional[torch.Tensor] = None     # int32 [max rows]
    ymap: Optional[torch.Tensor] = None     # int32 [max rows]
    mcount: Optional[torch.Tensor] = None   # int32 [1]


_WS = {}
_WS_OLD = []   # superseded workspaces stay alive: captured hipGraphs may still point at them


def _workspace(dev, n: int) -> torch.Tensor:
    """Split-K partial-slab workspace (64 MiB minimum; only grows, never freed)."""
    w = _WS.get(dev)
    if w is None or w.numel() < n:
        if w is not None:
            _WS_OLD.append(w)
        w = torch.empty(max(n, 16 << 20), dtype=torch.float32, device=dev)
        _WS[dev] = w
    return w


def dense_ok(segs: Sequence[Seg], M: int) -> bool:
    """May this launch run on the dense f16 GEMM (modes 4-6; the tuning table can still prefer the
    quantised kernel for the shape)?"""
    return M >= DENSE_MIN_M and all(s.w.d16 is not None and s.xmap is None and s.ymap is None for s in segs)


def _contiguous_cols(segs: Sequence[Seg]) -> bool:
    return all(s.ycol == segs[0].ycol + sum(x.w.rows for x in segs[:i]) for i, s in enumerate(segs))


def gemv_config(segs: Sequence[Seg], M: int):
    """(mode, waves, rt, ks) for a launch. mode 0 = waves split K (small batch, mapped rows);
    mode 1 = waves split rows over an LDS-staged activation tile (+ split-K across workgroups);
    mode 2 = large-M LDS-dequant GEMM (K-quants; rt = waves along M: 256- or 128-row blocks);
    mode 4/5 = large-M dense f16 GEMM on the weights' f16 copies, 128/256 weight rows per workgroup
    (rt as mode 2)."""
    from . import tuning
    if dense_ok(segs, M):
        cfg = tuning.select_dense(segs, M)
        if cfg is not None:
            return cfg
    return tuning.select(segs, M)


DENSE_MODES = (4, 5, 6, 10)


def _merge_dense(segs: Sequence[Seg]):
    """[d16 pointer, rows, K, ycol, seg] per launch segment: adjacent unmapped segments whose f16 copies are consecutive
    rows of one buffer (QWeight.expand_dense_group) and whose output columns are adjacent merge into one."""
    out = []
    for s in segs:
        if s.w.d16 is None:
            raise ValueError(f"{s.w.name}: dense modes {DENSE_MODES} need QWeight.expand_dense()")
        p = s.w.d16.data_ptr()
        plain = s.xmap is None and s.ymap is None and s.mcount is None
        if out and plain and out[-1][4].xmap is None and out[-1][4].ymap is None and out[-1][4].mcount is None:
            q, rows, K, ycol, s0 = out[-1]
            if K == s.w.K and q + rows * K * 2 == p and ycol + rows == s.ycol:
                out[-1] = [q, rows + s.w.rows, K, ycol, s0]
                continue
        out.append([p, s.w.rows, s.w.K, s.ycol, s])
    return out


def _seg_arr(segs: Sequence[Seg], mode: int):
    """ctypes segment list of a launch (pass len(arr) as the segment count): the dense modes point at the row-major
    f16 copies, adjacent copies of one buffer merged into one segment (_merge_dense); MoE row maps included (the
    dense GEMM gathers/scatters mapped rows like mode 2)."""
    if mode in DENSE_MODES:
        merged = _merge_dense(segs)
        arr = (_lib.NlsSeg * len(merged))()
        for i, (p, rows, K, ycol, s) in enumerate(merged):
            arr[i] = _lib.NlsSeg(p, _p(s.xmap), _p(s.ymap), _p(s.mcount), 1, rows, K, ycol)
        return arr
    arr = (_lib.NlsSeg * len(segs))()
    for i, s in enumerate(segs):
        arr[i] = _lib.NlsSeg(s.w.data.data_ptr(), _p(s.xmap), _p(s.ymap), _p(s.mcount), s.w.type, s.w.rows, s.w.K,
                             s.ycol)
    return arr


NORM_FUSE_LDS = 54 * 1024      # staged-row budget of the fused-norm GEMV (64 KiB LDS minus the reduce area)


def norm_fusable(M: int, K: int) -> bool:
    """Can a path-A GEMV fold the RMSNorm of its M input rows (K wide) into its activation staging?"""
    return M <= 16 and M * K * 2 <= NORM_FUSE_LDS


def qgemv(segs: Sequence[Seg], x: torch.Tensor, y: torch.Tensor, M: int, alpha: float = 1.0, epi: str = "f32",
          argmax: Optional[torch.Tensor] = None, waves: int = 0, rt: int = 1, mode: int = -1, ks: int = 1,
          norm=None, sel=None):
    """y (epilogue) alpha * x[:M] @ W^T for each segment. x: f16 [>=pad16(M), K].
    norm = (xf f32 [M, K], w f32 [K], eps[, ssq, ldss, nparts]): the GEMV input is f16(rmsnorm(xf) * w),
    computed inside the kernel (batch <= a few rows; `x` is then ignored on the GPU). With the partial
    sums of squares a qgemv_add_ssq producer left in `ssq`, the kernel skips the reduction pass and the
    tuned path-B (XL) config stays usable."""
    if norm is not None and x.is_cuda and len(norm) == 6 and norm[3] is not None:
        xf, nw, eps, ssq, ldss, nparts = norm
        if any(s.xmap is not None for s in segs) or M > 16:
            raise ValueError("fused-norm GEMV needs unmapped rows and M <= 16")
        cfg = gemv_config(segs, M)
        fz = _lib.NlsFuse(xf=xf.data_ptr(), ldxf=xf.stride(0), nw=nw.data_ptr(), eps=float(eps),
                          ssq_in=ssq.data_ptr(), ldss=int(ldss), nss_in=int(nparts))
        cands = [cfg] if cfg[0] in (0, 1) else []
        cands.append((0, 4, 2, 1))
        for mode, waves, rt, ks in cands:
            ws = None
            if mode == 1 and ks > 1:
                ws = _workspace(x.device, ks * M * sum(s.w.rows for s in segs)).data_ptr()
            rc = _lib.lib().nls_qgemv_ex(_segs(segs), len(segs), xf.data_ptr(), xf.stride(0), y.data_ptr(),
                                         y.stride(0), M, float(alpha), EPI[epi], _p(argmax), waves, rt, mode, ks, ws,
                                         _stream_ptr(xf), ctypes.byref(fz))
            if rc == 0:
                return y
            if rc != -1:
                _lib.check(rc, "nls_qgemv_ex(norm)")
        raise ValueError("no launch config takes the split-RMSNorm operands")
    if norm is not None and x.is_cuda:
        xf, nw, eps = norm[:3]
        if any(s.xmap is not None for s in segs) or not norm_fusable(M, segs[0].w.K):
            raise ValueError("fused-norm GEMV needs unmapped rows and M*K*2 <= NORM_FUSE_LDS")
        mode, waves, rt, ks = gemv_config(segs, M)
        if mode != 0:
            waves, rt = 4, 2
        arr = (_lib.NlsSeg * len(segs))()
        for i, s in enumerate(segs):
            arr[i] = _lib.NlsSeg(s.w.data.data_ptr(), None, None, None, s.w.type, s.w.rows, s.w.K, s.ycol)
        _lib.check(_lib.lib().nls_qgemv_norm(arr, len(segs), xf.data_ptr(), xf.stride(0), nw.data_ptr(), float(eps),
                                             y.data_ptr(), y.stride(0), M, float(alpha), EPI[epi], _p(argmax), waves,
                                             rt, _stream_ptr(xf)), "nls_qgemv_norm")
        return y
    if norm is not None:
        xf, nw, eps = norm[:3]
        xs = xf[:M].float()
        x = (xs * torch.rsqrt(xs.pow(2).mean(dim=1, keepdim=True) + eps) * nw.float()).to(ACT_DTYPE)
    if x.is_cuda and sel is not None:
        # MoE decode with few tokens: launch only the routed experts' tiles (path A, mapped rows).
        # sel = (int32 slots tensor, n_slots, base): slot i serves segment sel[i] - base.
        if x.dtype != ACT_DTYPE:
            raise TypeError(f"qgemv: activations must be {ACT_DTYPE}, got {x.dtype}")
        st, nslots, base = sel
        mode, waves, rt, ks = MOE_GEMV if mode < 0 or waves == 0 else (mode, waves, rt, ks)
        fz = _lib.NlsFuse(sel=st.data_ptr(), sel_slots=int(nslots), sel_base=int(base))
        _lib.check(_lib.lib().nls_qgemv_ex(_segs(segs), len(segs), x.data_ptr(), x.stride(0), y.data_ptr(),
                                           y.stride(0), M, float(alpha), EPI[epi], _p(argmax), waves, rt, 0, 1, None,
                                           _stream_ptr(x), ctypes.byref(fz)), "nls_qgemv_ex(sel)")
        return y
    if x.is_cuda:
        if x.dtype != ACT_DTYPE:
            raise TypeError(f"qgemv: activations must be {ACT_DTYPE}, got {x.dtype}")
        L = _lib.lib()
        mapped = any(s.xmap is not None for s in segs)
        if not mapped and (x.shape[0] < M or (epi != "argmax" and y.shape[0] < M)):
            # the kernels index rows 0..M-1 unchecked: fail here, not with a device fault
            raise ValueError(f"qgemv: M={M} rows but x has {x.shape[0]}, y {y.shape[0]}")
        if mode < 0 or waves == 0:
            mode, waves, rt, ks = gemv_config(segs, M) if not mapped else MOE_GEMV
        if M > 64 and mode == 0:
            # mapped (MoE) rows / path A: chunks of 64 rows
            for m0 in range(0, M, 64):
                mm = min(64, M - m0)
                qgemv(segs, x[m0:], y[m0:], mm, alpha, epi, None if argmax is None else argmax[m0:], waves, rt,
                      mode, ks)
            return y
        arr = _seg_arr(segs, mode)
        ws = None
        if mode != 0 and ks > 1:
            width = segs[0].w.rows if mapped else sum(s.w.rows for s in segs)   # mapped split-K: shared columns
            ws = _workspace(x.device, ks * M * width).data_ptr()
        rc = L.nls_qgemv(arr, len(arr), x.data_ptr(), x.stride(0), y.data_ptr(), y.stride(0), M, float(alpha),
                         EPI[epi], _p(argmax), waves, rt, mode, ks, ws, _stream_ptr(x))
        _lib.check(rc, "nls_qgemv")
        return y
    # ---- CPU reference ----
    for s in segs:
        W = s.w.dense()
        if s.xmap is not None:
            cnt = int(s.mcount.item()) if s.mcount is not None else M
            cnt = min(cnt, M)
            xi = s.xmap[:cnt].long()
            yi = s.ymap[:cnt].long() if s.ymap is not None else torch.arange(cnt)
            xs = x.index_select(0, xi).float()
        else:
            cnt = M
            xs = x[:M].float()
            yi = torch.arange(M)
        if cnt == 0:
            continue
        acc = alpha * (xs @ W.t())
        n = W.shape[0]
        if epi == "swiglu":
            a4 = acc.view(cnt, n // 16, 2, 8)
            g, u = a4[:, :, 0, :], a4[:, :, 1, :]
            out = (torch.nn.functional.silu(g) * u).reshape(cnt, n // 2)
            y[yi, s.ycol:s.ycol + n // 2] = out.to(y.dtype)
        elif epi == "add":
            y[yi, s.ycol:s.ycol + n] += acc.to(y.dtype)
        elif epi != "argmax":
            y[yi, s.ycol:s.ycol + n] = acc.to(y.dtype)
        if argmax is not None:
            v, idx = acc.max(dim=1)
            key = _argmax_keys(v, idx + s.ycol)
            argmax[yi] = torch.maximum(argmax[yi], key)
    return y


def qgemv_add_ssq(seg: Seg, xin: torch.Tensor, x: torch.Tensor, M: int, alpha: float, ssq: torch.Tensor,
                  ldss: int, cfg=None) -> Optional[int]:
    """x[:M] += alpha * xin @ W^T, and when the launch runs on path A, each workgroup also leaves its
    share of sum(x_new^2) per token in ssq[m * ldss + wg] for the next fused-norm GEMV (split RMSNorm:
    no norm launch, no reduction pass in the consumer). Returns the number of shares, or None when
    this launch cannot produce them (the consumer then normalises from the full rows)."""
    if x.is_cuda and seg.xmap is None and M <= 32:
        mode, waves, rt, ks = cfg or gemv_config([seg], M)
        ntile = -(-seg.w.rows // (16 * rt))
        if mode == 0 and ntile <= ldss:
            fz = _lib.NlsFuse(ssq_out=ssq.data_ptr(), ldss=int(ldss))
            rc = _lib.lib().nls_qgemv_ex(_segs([seg]), 1, xin.data_ptr(), xin.stride(0), x.data_ptr(), x.stride(0), M,
                                         float(alpha), EPI["add"], None, waves, rt, 0, 1, None, _stream_ptr(x),
                                         ctypes.byref(fz))
            if rc == 0:
                return ntile
            if rc != -1:
                _lib.check(rc, "nls_qgemv_ex(ssq)")
    qgemv([seg], xin, x, M, alpha=alpha, epi="add")
    return None


def _segs(segs: Sequence[Seg]):
    arr = (_lib.NlsSeg * len(segs))()
    for i, s in enumerate(segs):
        arr[i] = _lib.NlsSeg(s.w.data.data_ptr(), _p(s.xmap), _p(s.ymap), _p(s.mcount), s.w.type, s.w.rows, s.w.K,
                             s.ycol)
    return arr


def qgemv_add_rmsnorm(seg: Seg, xin: torch.Tensor, x: torch.Tensor, norm_w: torch.Tensor, h: torch.Tensor, M: int,
                      alpha: float, eps: float, cfg=None, counter: Optional[torch.Tensor] = None):
    """x[:M] += alpha * xin @ W^T, then h[:M] = rmsnorm(x[:M]) * norm_w (f16). With a split-K
    launch config the partial slabs are reduced by the fused reduce+residual+RMSNorm kernel; a few-row
    path-A launch (M <= ADDNORM_MAX_M, `counter`: a zeroed int32 device word) normalises in its last
    workgroup, so the norm costs no launch at all."""
    if x.is_cuda and seg.xmap is None:
        mode, waves, rt, ks = cfg or gemv_config([seg], M)
        if (mode == 0 and counter is not None and M <= ADDNORM_MAX_M and seg.ycol == 0
                and seg.w.rows == x.shape[1]):
            fz = _lib.NlsFuse(hout=h.data_ptr(), ldh=h.stride(0), onw=norm_w.data_ptr(), cnt=counter.data_ptr(),
                              eps=float(eps))
            _lib.check(_lib.lib().nls_qgemv_ex(_segs([seg]), 1, xin.data_ptr(), xin.stride(0), x.data_ptr(),
                                               x.stride(0), M, float(alpha), EPI["add"], None, waves, rt, 0, 1, None,
                                               _stream_ptr(x), ctypes.byref(fz)), "nls_qgemv_ex(addnorm)")
            return h
        if mode != 0 and ks > 1 and seg.ycol == 0 and seg.w.rows == x.shape[1]:
            L = _lib.lib()
            ws = _workspace(x.device, ks * M * seg.w.rows)
            arr = _seg_arr([seg], mode)
            st = _stream_ptr(x)
            _lib.check(L.nls_qgemv(arr, 1, xin.data_ptr(), xin.stride(0), x.data_ptr(), x.stride(0), M, float(alpha),
                                   EPI["slabs"], None, waves, rt, mode, ks, ws.data_ptr(), st), "nls_qgemv")
            _lib.check(L.nls_splitk_add_rmsnorm(ws.data_ptr(), ks, M, float(alpha), x.data_ptr(), x.stride(0),
                                                norm_w.data_ptr(), h.data_ptr(), h.stride(0), x.shape[1], float(eps),
                                                st), "nls_splitk_add_rmsnorm")
            return h
    if cfg is not None and x.is_cuda:
        mode, waves, rt, ks = cfg
        qgemv([seg], xin, x, M, alpha=alpha, epi="add", mode=mode, waves=waves, rt=rt, ks=ks)
    else:
        qgemv([seg], xin, x, M, alpha=alpha, epi="add")
    return rmsnorm(x, norm_w, h, M, eps)


def qgemv_add_norm_route(seg: Seg, xin: torch.Tensor, x: torch.Tensor, nw: torch.Tensor, h: torch.Tensor, M: int,
                         alpha: float, eps: float, counter: torch.Tensor, wr: torch.Tensor, logits: torch.Tensor, k: int,
                         topw: torch.Tensor, counts: torch.Tensor, xrows: torch.Tensor, yrows: torch.Tensor, cap: int,
                         renorm: bool = True, sel: Optional[torch.Tensor] = None) -> bool:
    """MoE decode (M <= 4 tokens): the o projection x[:M] += alpha * xin @ W^T, then -- in its last workgroup --
    the FFN RMSNorm h = f16(rmsnorm(x) * nw), the router logits h @ wr^T and the top-k route (moe_route): the
    separate norm + router + route launch (moe_norm_route) folded into the projection. False (nothing done)
    where the fused launch does not apply; the caller then runs the two launches."""
    if not x.is_cuda or seg.xmap is not None or seg.ycol or seg.w.rows != x.shape[1] or M > 4:
        return False
    mode, waves, rt, ks = gemv_config([seg], M)
    if mode != 0:
        mode, waves, rt, ks = 0, 4, 1, 1
    fz = _lib.NlsFuse(hout=h.data_ptr(), ldh=h.stride(0), onw=nw.data_ptr(), cnt=counter.data_ptr(), eps=float(eps),
                      wr=wr.data_ptr(), E=int(wr.shape[0]), topk=int(k), renorm=int(renorm), rcap=int(cap),
                      rlogits=logits.data_ptr(), topw=topw.data_ptr(), counts=counts.data_ptr(),
                      xrows=xrows.data_ptr(), yrows=yrows.data_ptr(), rsel=_p(sel))
    rc = _lib.lib().nls_qgemv_ex(_segs([seg]), 1, xin.data_ptr(), xin.stride(0), x.data_ptr(), x.stride(0), M,
                                 float(alpha), EPI["add"], None, waves, rt, 0, 1, None, _stream_ptr(x), ctypes.byref(fz))
    if rc == -1:
        return False
    _lib.check(rc, "nls_qgemv_ex(add+norm+route)")
    return True


def _argmax_keys(v: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    u = v.float().view(torch.int32).long() & 0xFFFFFFFF
    neg = (u & 0x80000000) != 0
    u = torch.where(neg, (~u) & 0xFFFFFFFF, u | 0x80000000)
    # GPU keys are unsigned u64; on CPU flip the top bit so signed int64 order == unsigned order
    return ((u ^ 0x80000000) << 32) | (0xFFFFFFFF - idx.long())


def argmax_reset(keys: torch.Tensor):
    """Initial value of a fused-argmax key buffer (smaller than every key). Decode on one GPU re-arms the
    keys inside argmax_unpack(rearm=True) instead of a separate launch (LlamaModel._keys_clean)."""
    if keys.is_cuda:
        keys.zero_()
    else:
        keys.fill_(torch.iinfo(torch.int64).min)


# ---------------------------------------------------------------------------
# Normalisation, RoPE + KV append, embedding, attention, sampling, MoE routing
# ---------------------------------------------------------------------------

def rmsnorm(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, M: int, eps: float):
    D = x.shape[1]
    if x.is_cuda:
        _lib.check(_lib.lib().nls_rmsnorm(x.data_ptr(), x.stride(0), w.data_ptr(), out.data_ptr(), out.stride(0), M,
                                          D, float(eps), int(out.dtype == torch.float32), _stream_ptr(x)),
                   "nls_rmsnorm")
        return out
    xs = x[:M].float()
    r = xs * torch.rsqrt(xs.pow(2).mean(dim=1, keepdim=True) + eps) * w.float()
    out[:M] = r.to(out.dtype)
    return out


def rope_inv_freq(head_dim: int, base: float, freq_factors=None) -> np.ndarray:
    """theta_i = base^(-2i/D), divided by GGUF `rope_freqs.weight` when present (Llama-3.1+ long-context
    frequency scaling, llama.cpp `rope_freq_factors`)."""
    inv = 1.0 / (base ** (np.arange(0, head_dim, 2, dtype=np.float64) / head_dim))
    if freq_factors is not None:
        inv = inv / np.asarray(freq_factors, dtype=np.float64).reshape(-1)[:head_dim // 2]
    return inv


def rope_table(max_pos: int, head_dim: int, base: float, device, freq_factors=None,
               pos_scale: float = 1.0) -> torch.Tensor:
    """[max_pos, D/2, 2] (cos, sin). `pos_scale` < 1: linear RoPE scaling (`rope.scaling.type=linear`)."""
    inv = rope_inv_freq(head_dim, base, freq_factors)
    ang = (np.arange(max_pos, dtype=np.float64) * pos_scale)[:, None] * inv[None, :]
    cs = np.stack([np.cos(ang), np.sin(ang)], axis=-1).astype(np.float32)   # [P, D/2, 2]
    return torch.from_numpy(cs).to(device)


# K/V cache element types: bf16, or OCP fp8 e4m3 (half the attention bytes per decode step; opt-in,
# NLS_KV_DTYPE=fp8 -- the kernels saturate to +-448 and convert exactly to bf16 on load)
KV_DTYPES = {"bf16": torch.bfloat16, "fp8": torch.float8_e4m3fn}


def _kv_fn(name: str, kc: torch.Tensor):
    """The kernel entry point for this cache's element type (`<name>8`: fp8)."""
    if kc.dtype == torch.float8_e4m3fn:
        return getattr(_lib.lib(), name + "8")
    if kc.dtype != torch.bfloat16:
        raise TypeError(f"{name}: KV cache dtype {kc.dtype} (bf16 or float8_e4m3fn)")
    return getattr(_lib.lib(), name)


def rope_kv(qkv: torch.Tensor, pos: torch.Tensor, slot: torch.Tensor, cs: torch.Tensor, q_out: torch.Tensor,
            kc: torch.Tensor, vc: torch.Tensor, T: int, Hq: int, Hkv: int, D: int, neox: bool = False,
            bias: Optional[torch.Tensor] = None):
    """kc/vc: [slots, Hkv, D] bf16 for one layer. slot (int32) < 0 skips the cache write.
    `bias` (f32 [(Hq+2*Hkv)*D], Qwen2 QKV bias) is added before the rotation."""
    if qkv.is_cuda:
        _lib.check(_kv_fn("nls_rope_kv", kc)(qkv.data_ptr(), qkv.stride(0), 1, 0, _p(bias), pos.data_ptr(),
                                          slot.data_ptr(), cs.data_ptr(), q_out.data_ptr(), q_out.stride(0),
                                          kc.data_ptr(), vc.data_ptr(), T, Hq, Hkv, D, int(neox), _stream_ptr(qkv)),
                   "nls_rope_kv")
        return
    x = qkv[:T].float()
    if bias is not None:
        x = x + bias.float()[None, :x.shape[1]]
    p = pos[:T].long()
    c, s = cs[p, :, 0], cs[p, :, 1]                      # [T, D/2]

    def rot(h):                                          # h: [T, H, D]
        if neox:
            x0, x1 = h[..., :D // 2], h[..., D // 2:]
        else:
            x0, x1 = h[..., 0::2], h[..., 1::2]
        cc, ss = c[:, None, :], s[:, None, :]
        y0, y1 = x0 * cc - x1 * ss, x0 * ss + x1 * cc
        if neox:
            return torch.cat([y0, y1], dim=-1)
        return torch.stack([y0, y1], dim=-1).flatten(-2)

    q = rot(x[:, :Hq * D].view(T, Hq, D))
    k = rot(x[:, Hq * D:(Hq + Hkv) * D].view(T, Hkv, D))
    v = x[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].view(T, Hkv, D)
    q_out[:T, :Hq * D] = q.reshape(T, Hq * D).to(q_out.dtype)
    sl = slot[:T].long()
    ok = sl >= 0
    kc[sl[ok]] = k[ok].to(kc.dtype)
    vc[sl[ok]] = v[ok].to(vc.dtype)


def qkv_rope_kv(segs: Sequence[Seg], h: torch.Tensor, qkv: torch.Tensor, pos: torch.Tensor, slot: torch.Tensor,
                cs: torch.Tensor, q_out: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, T: int, Hq: int, Hkv: int,
                D: int, neox: bool = False, cfg=None, bias: Optional[torch.Tensor] = None, norm=None,
                fuse_rope: bool = True):
    """QKV projection + RoPE + paged KV append. A path-A (few-row) launch rotates in the GEMV epilogue
    and writes q / K / V directly (one launch); with a split-K launch config the partial slabs are
    summed inside the RoPE kernel (no separate reduce pass, no fp32 qkv round trip)."""
    if h.is_cuda and all(s.xmap is None for s in segs):
        mode, waves, rt, ks = cfg or gemv_config(segs, T)
        ncol = sum(s.w.rows for s in segs)
        contiguous = all(s.ycol == sum(x.w.rows for x in segs[:i]) for i, s in enumerate(segs))
        if (mode == 0 and T <= 64 and not neox and contiguous and ncol == (Hq + 2 * Hkv) * D and fuse_rope
                and kc.dtype == torch.bfloat16):
            # path A: RoPE + KV append in the GEMV epilogue (no qkv round trip, no RoPE launch)
            fz = _lib.NlsFuse(pos=pos.data_ptr(), slot=slot.data_ptr(), cs=cs.data_ptr(), bias=_p(bias),
                              q_out=q_out.data_ptr(), ldq=q_out.stride(0), kc=kc.data_ptr(), vc=vc.data_ptr(),
                              Hq=Hq, Hkv=Hkv, D=D)
            if norm is not None:
                xf, nw, eps = norm[:3]
                if not norm_fusable(T, segs[0].w.K):
                    raise ValueError("fused-norm GEMV needs M*K*2 <= NORM_FUSE_LDS")
                fz.xf, fz.ldxf, fz.nw, fz.eps = xf.data_ptr(), xf.stride(0), nw.data_ptr(), float(eps)
                if len(norm) == 6 and norm[3] is not None:
                    fz.ssq_in, fz.ldss, fz.nss_in = norm[3].data_ptr(), int(norm[4]), int(norm[5])
            _lib.check(_lib.lib().nls_qgemv_ex(_segs(segs), len(segs), h.data_ptr(), h.stride(0), qkv.data_ptr(),
                                               qkv.stride(0), T, 1.0, EPI["rope"], None, waves, rt, 0, 1, None,
                                               _stream_ptr(h), ctypes.byref(fz)), "nls_qgemv_ex(rope)")
            return
    if h.is_cuda and all(s.xmap is None for s in segs) and norm is None:
        mode, waves, rt, ks = cfg or gemv_config(segs, T)
        ncol = sum(s.w.rows for s in segs)
        contiguous = all(s.ycol == sum(x.w.rows for x in segs[:i]) for i, s in enumerate(segs))
        if (mode in (4, 5, 10) and ks == 1 and contiguous and ncol == (Hq + 2 * Hkv) * D
                and not neox and fuse_rope and kc.dtype == torch.bfloat16):
            # large-M GEMM on the dense f16 copies with RoPE + KV append in its epilogue (no f32 qkv round trip,
            # no RoPE launch)
            fz = _lib.NlsFuse(pos=pos.data_ptr(), slot=slot.data_ptr(), cs=cs.data_ptr(), bias=_p(bias),
                              q_out=q_out.data_ptr(), ldq=q_out.stride(0), kc=kc.data_ptr(), vc=vc.data_ptr(),
                              Hq=Hq, Hkv=Hkv, D=D)
            arr = _seg_arr(segs, mode)
            _lib.check(_lib.lib().nls_qgemv_ex(arr, len(arr), h.data_ptr(), h.stride(0),
                                               qkv.data_ptr(), qkv.stride(0), T, 1.0, EPI["rope"], None, waves, rt,
                                               mode, 1, None, _stream_ptr(h), ctypes.byref(fz)),
                       "nls_qgemv_ex(dense rope)")
            return
        if mode != 0 and ks > 1 and contiguous and ncol == (Hq + 2 * Hkv) * D:
            L = _lib.lib()
            ws = _workspace(h.device, ks * T * ncol)
            arr = _seg_arr(segs, mode)
            st = _stream_ptr(h)
            _lib.check(L.nls_qgemv(arr, len(arr), h.data_ptr(), h.stride(0), qkv.data_ptr(), qkv.stride(0), T, 1.0,
                                   EPI["slabs"], None, waves, rt, mode, ks, ws.data_ptr(), st), "nls_qgemv")
            _lib.check(_kv_fn("nls_rope_kv", kc)(ws.data_ptr(), ncol, ks, T * ncol, _p(bias), pos.data_ptr(),
                                                 slot.data_ptr(),
                                     cs.data_ptr(), q_out.data_ptr(), q_out.stride(0), kc.data_ptr(), vc.data_ptr(),
                                     T, Hq, Hkv, D, int(neox), st), "nls_rope_kv")
            return
    qgemv(segs, h, qkv, T, norm=norm)
    rope_kv(qkv, pos, slot, cs, q_out, kc, vc, T, Hq, Hkv, D, neox, bias)


def embed(ids: torch.Tensor, w: QWeight, out: torch.Tensor, T: int, scale: float = 1.0, prev=None):
    """out[:T] = scale * W[ids[:T]]. prev = (next_ids, use_prev) (chained decode): first
    ids[t] = next_ids[t] where use_prev[t] != 0 (in the same launch on the GPU)."""
    if ids.is_cuda:
        if prev is not None:
            nxt, use = prev
            _lib.check(_lib.lib().nls_embed_prev(ids.data_ptr(), nxt.data_ptr(), use.data_ptr(), T, w.data.data_ptr(),
                                                 w.type, w.rows, w.K, out.data_ptr(), out.stride(0), float(scale),
                                                 _stream_ptr(ids)), "nls_embed_prev")
            return out
        _lib.check(_lib.lib().nls_embed(ids.data_ptr(), T, w.data.data_ptr(), w.type, w.rows, w.K, out.data_ptr(),
                                        out.stride(0), float(scale), _stream_ptr(ids)), "nls_embed")
        return out
    if prev is not None:
        nxt, use = prev
        torch.where(use[:T] != 0, nxt[:T], ids[:T], out=ids[:T])
    out[:T] = scale * w.dense()[ids[:T].long()]
    return out


def attention(q: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, block_tables: torch.Tensor,
              tok_seq: torch.Tensor, ctx_len: torch.Tensor, out: torch.Tensor, T: int, Hq: int, Hkv: int, D: int,
              block_size: int, scale: float, chunk: int = 256, n_split: int = 1,
              workspace: Optional[torch.Tensor] = None, counters: Optional[torch.Tensor] = None):
    """Paged GQA attention; query t attends to the first ctx_len[t] positions of sequence tok_seq[t].
    n_split > 1 (flash-decoding): `counters` (zeroed int32 [>= T*Hkv]) lets the last split of each
    (token, kv head) merge the partials in-kernel; without it a combine kernel runs."""
    if q.is_cuda:
        po = pml = None
        if counters is not None and (counters.numel() < T * Hkv or counters.dtype != torch.int32):
            raise ValueError("attention counters must be int32 with >= T*Hkv entries")
        if n_split > 1:
            need = T * Hq * n_split * (D + 2)
            if workspace is None or workspace.numel() < need:
                workspace = torch.empty(need, dtype=torch.float32, device=q.device)
            po = workspace.data_ptr()
            pml = po + T * Hq * n_split * D * 4
        _lib.check(_kv_fn("nls_attn_decode", kc)(q.data_ptr(), q.stride(0), kc.data_ptr(), vc.data_ptr(),
                                              block_tables.data_ptr(), block_tables.stride(0), tok_seq.data_ptr(),
                                              ctx_len.data_ptr(), T, Hq, Hkv, D, block_size, float(scale), chunk,
                                              n_split, out.data_ptr(), out.stride(0), po, pml,
                                              _p(counters) if n_split > 1 else None, _stream_ptr(q)),
                   "nls_attn_decode")
        return out
    G = Hq // Hkv
    for t in range(T):
        n = int(ctx_len[t])
        if n <= 0:
            out[t, :Hq * D] = 0
            continue
        bt = block_tables[int(tok_seq[t])].long()
        p = torch.arange(n)
        slots = bt[p // block_size] * block_size + p % block_size
        k = kc[slots].float()                                  # [n, Hkv, D]
        v = vc[slots].float()
        qq = q[t, :Hq * D].float().view(Hkv, G, D)
        s = torch.einsum("hgd,nhd->hgn", qq, k) * scale
        pr = torch.softmax(s, dim=-1)
        o = torch.einsum("hgn,nhd->hgd", pr, v)
        out[t, :Hq * D] = o.reshape(Hq * D).to(out.dtype)
    return out


# attn_prefill.hip: the 8-wave 32x32x16 kernel takes 64-token query blocks; NLS_PREFILL_V1=1 selects the first
# kernel (4 waves, 32-token blocks) for A/B
PREFILL_V1 = _os.environ.get("NLS_PREFILL_V1", "0") == "1"
PREFILL_QT = 32 if PREFILL_V1 else 64      # tokens per attention_prefill query block


def prefill_blocks(tok_seq, pos, T: int):
    """Query blocks for attention_prefill: (t0, ntok<=PREFILL_QT, seq, pos0) over runs of consecutive
    tokens of one sequence (numpy int arrays in, int32 [nqb, 4] out)."""
    ts = np.asarray(tok_seq[:T])
    ps = np.asarray(pos[:T])
    if T == 0:
        return np.zeros((0, 4), np.int32)
    cut = np.flatnonzero((ts[1:] != ts[:-1]) | (ps[1:] != ps[:-1] + 1)) + 1
    starts = np.concatenate([[0], cut])
    ends = np.concatenate([cut, [T]])
    out = []
    for a, b in zip(starts, ends):
        for t in range(a, b, PREFILL_QT):
            out.append((t, min(PREFILL_QT, b - t), ts[a], ps[t]))
    return np.asarray(out, dtype=np.int32).reshape(-1, 4)


def attention_prefill_ok(Hq: int, Hkv: int, D: int) -> bool:
    return Hq % Hkv == 0 and (Hq // Hkv) % 4 == 0 and D in (64, 128)


def attention_prefill(q: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, block_tables: torch.Tensor,
                      qblocks: torch.Tensor, nqb: int, tok_seq: torch.Tensor, ctx_len: torch.Tensor,
                      out: torch.Tensor, T: int, Hq: int, Hkv: int, D: int, block_size: int, scale: float):
    """Causal MFMA flash attention over the paged cache for prompt chunks (query blocks of PREFILL_QT tokens,
    ops.prefill_blocks)."""
    if q.is_cuda:
        _lib.check(_kv_fn("nls_attn_prefill_v1" if PREFILL_V1 else "nls_attn_prefill", kc)(q.data_ptr(), q.stride(0), kc.data_ptr(), vc.data_ptr(),
                                               block_tables.data_ptr(), block_tables.stride(0), qblocks.data_ptr(),
                                               nqb, Hq, Hkv, D, block_size, float(scale), out.data_ptr(),
                                               out.stride(0), _stream_ptr(q)), "nls_attn_prefill")
        return out
    return attention(q, kc, vc, block_tables, tok_seq, ctx_len, out, T, Hq, Hkv, D, block_size, scale)


def argmax(logits: torch.Tensor, M: int, out: torch.Tensor):
    V = logits.shape[1]
    if logits.is_cuda:
        _lib.check(_lib.lib().nls_argmax(logits.data_ptr(), logits.stride(0), M, V, out.data_ptr(),
                                         _stream_ptr(logits)), "nls_argmax")
        return out
    out[:M] = logits[:M].float().argmax(dim=1).to(out.dtype)
    return out


def topc_candidates(logits: torch.Tensor, n: int, C: int, vocab_lo: int, valid: int):
    """Per row, the C largest logits of a vocab shard (columns [0, valid) of `logits`; the rest are padding)
    in increasing vocabulary order: (values f32 [n, C], global token ids int32 [n, C]), padded with
    (-inf, -1) where the shard holds fewer than C tokens. Tensor-parallel sampling gathers these instead of
    the [n, vocab] logits (engine: _gather / _sample_candidates).

    GPU: ONE launch of sample.hip topc_kernel (radix select + in-order compaction) writing both planes of a
    [2, n, C] int32 block -- the source buffer of the candidate all-gather, which comm.gather_candidates uses as it
    is (`_packed`): no topk / sort / gather / fill / stack kernels in the captured decode graph."""
    if logits.is_cuda:
        if logits.dtype != torch.float32 or logits.stride(1) != 1:
            raise TypeError("topc_candidates: fp32 row-major logits")
        src = torch.empty(2, n, C, dtype=torch.int32, device=logits.device)
        _lib.check(_lib.lib().nls_topc(logits.data_ptr(), logits.stride(0), n, int(valid), C, int(vocab_lo),
                                       src.data_ptr(), _stream_ptr(logits)), "nls_topc")
        v, i = src[0].view(torch.float32), src[1]
        v._packed = i._packed = src
        return v, i
    k = max(0, min(C, valid))
    v = torch.full((n, C), float("-inf"), dtype=torch.float32, device=logits.device)
    i = torch.full((n, C), -1, dtype=torch.int32, device=logits.device)
    if k and n:
        tv, ti = torch.topk(logits[:n, :valid].float(), k, dim=1)
        ti, order = torch.sort(ti, dim=1)                    # vocabulary order within the shard
        v[:, :k] = torch.gather(tv, 1, order)
        i[:, :k] = (ti + vocab_lo).to(torch.int32)
    return v, i


def argmax_unpack(keys: torch.Tensor, n: int, out: torch.Tensor, rearm: bool = False):
    """Token ids from the fused arg-max keys. rearm: reset keys[:n] in the same launch (see argmax_reset)."""
    if keys.is_cuda:
        fn = _lib.lib().nls_argmax_unpack_rearm if rearm else _lib.lib().nls_argmax_unpack
        _lib.check(fn(keys.data_ptr(), n, out.data_ptr(), _stream_ptr(keys)), "nls_argmax_unpack")
        return out
    out[:n] = (0xFFFFFFFF - (keys[:n] & 0xFFFFFFFF)).to(out.dtype)
    if rearm:
        argmax_reset(keys[:n])
    return out


SAMPLE_PARAMS_BYTES = 40      # csrc/kernels/sample.hip SampleParams


def sample_params_bytes(p=None) -> bytes:
    """Device SampleParams of one row; None: a greedy row (skipped by the in-graph sampler)."""
    if p is None:
        sp = _lib.SampleParams(0.0, 1.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0, 0, 0)
    else:
        sp = _lib.SampleParams(p.temperature, p.top_p, p.min_p, p.repeat_penalty, p.presence_penalty,
                               p.frequency_penalty, 0.0, int(p.top_k or 0), 0, 0)
    raw = bytes(sp)
    assert len(raw) == SAMPLE_PARAMS_BYTES
    return raw


def sample_decode(logits: torch.Tensor, n: int, params: torch.Tensor, seeds: torch.Tensor, pos: torch.Tensor,
                  ctx_len: torch.Tensor, hist: torch.Tensor, next_ids: torch.Tensor):
    """In-graph sampling of decode rows [0, n): rows whose device params ask for sampling overwrite
    next_ids with a draw (uniform from (seed, position)), appending it to their history ring."""
    if logits.dtype != torch.float32 or logits.stride(1) != 1:
        raise TypeError("sample_decode: fp32 row-major logits")
    _lib.check(_lib.lib().nls_sample_decode(logits.data_ptr(), logits.stride(0), n, logits.shape[1], params.data_ptr(),
                                            seeds.data_ptr(), pos.data_ptr(), ctx_len.data_ptr(), hist.data_ptr(),
                                            hist.shape[1], next_ids.data_ptr(), _stream_ptr(logits)),
               "nls_sample_decode")


def sample_decode_cand(vals: torch.Tensor, ids: torch.Tensor, n: int, params: torch.Tensor, seeds: torch.Tensor,
                       pos: torch.Tensor, ctx_len: torch.Tensor, hist: torch.Tensor, next_ids: torch.Tensor):
    """In-graph sampling of tensor-parallel decode rows [0, n) from the gathered candidates (values `vals`
    [n, M] in vocabulary order -- scratch, penalties are applied in place -- and global ids `ids` [n, M]):
    sample_decode's semantics with the history ring mapped onto candidate positions."""
    M = vals.shape[1]
    if vals.is_cuda:
        if vals.dtype != torch.float32 or vals.stride(1) != 1 or ids.stride(1) != 1:
            raise TypeError("sample_decode_cand: fp32 / int32 row-major candidates")
        _lib.check(_lib.lib().nls_sample_decode_cand(vals.data_ptr(), vals.stride(0), n, M, ids.data_ptr(),
                                                     ids.stride(0), params.data_ptr(), seeds.data_ptr(), pos.data_ptr(),
                                                     ctx_len.data_ptr(), hist.data_ptr(), hist.shape[1],
                                                     next_ids.data_ptr(), _stream_ptr(vals)), "nls_sample_decode_cand")
        return
    # CPU twin of sample.hip sample_decode_cand_kernel (gloo rehearsals of the tensor-parallel path)
    from ..engine.sampling import SamplingParams, sample_rows, uniform01
    raw = params.cpu().numpy()
    S = hist.shape[1]
    for r in range(n):
        if int(ctx_len[r]) <= 0:
            continue
        sp = _lib.SampleParams.from_buffer_copy(raw[r].tobytes())
        p = SamplingParams(temperature=sp.temperature, top_k=sp.top_k, top_p=sp.top_p, min_p=sp.min_p,
                           repeat_penalty=sp.repeat_penalty, presence_penalty=sp.presence_penalty,
                           frequency_penalty=sp.frequency_penalty)
        if p.greedy:
            continue
        ps = int(pos[r])
        nh = min(S, ps + 1)
        idl = ids[r].tolist()
        at = {t: j for j, t in enumerate(idl) if t >= 0}
        hp = [at[t] for t in hist[r, :nh].tolist() if t in at]
        seed = int(seeds[r]) & 0xFFFFFFFFFFFFFFFF
        j = sample_rows(vals[r:r + 1].float(), [p], [hp], [uniform01(seed, ps)])[0]
        tok = idl[j] if 0 <= j < M and idl[j] >= 0 else 0
        next_ids[r] = tok
        hist[r, (ps + 1) % S] = tok


def moe_norm_route(x: torch.Tensor, nw: torch.Tensor, eps: float, wr: torch.Tensor, h: torch.Tensor,
                   logits: torch.Tensor, T: int, k: int, topw: torch.Tensor, counts: torch.Tensor, xrows: torch.Tensor,
                   yrows: torch.Tensor, cap: int, renorm: bool = True, sel: Optional[torch.Tensor] = None) -> bool:
    """h[:T] = rmsnorm(x[:T]) * nw (f16), router logits h @ wr^T (wr: the router's f16 copy [E, D]) and the
    top-k route, in one launch on the GPU (T <= 4, E in {2, 4, 8}). Returns False, having done nothing,
    when the fused kernel does not take the shape."""
    E = wr.shape[0]
    if x.is_cuda:
        rc = _lib.lib().nls_moe_norm_route(x.data_ptr(), x.stride(0), nw.data_ptr(), float(eps), x.shape[1],
                                           wr.data_ptr(), h.data_ptr(), h.stride(0), logits.data_ptr(), T, E, k,
                                           int(renorm), topw.data_ptr(), counts.data_ptr(), xrows.data_ptr(),
                                           yrows.data_ptr(), cap, _p(sel), _stream_ptr(x))
        if rc == -1:
            return False
        _lib.check(rc, "nls_moe_norm_route")
        return True
    rmsnorm(x, nw, h, T, eps)
    logits[:T] = h[:T].float() @ wr.float().t()
    moe_route(logits, T, k, topw, counts, xrows, yrows, cap, renorm, sel)
    return True


def router_logits(h: torch.Tensor, wr: torch.Tensor, logits: torch.Tensor, T: int,
                  zero: Optional[torch.Tensor] = None) -> torch.Tensor:
    """logits[:T] = h[:T] @ wr^T for a MoE router (wr: its f16 copy [E, D], E in {2, 4, 8}): one launch of
    T / 4 workgroups (ops.hip router_logits_kernel) instead of a GEMM tiled for 128-row weight blocks.
    `zero` (int32, optional): zeroed in the same launch (the next moe_route's expert counts)."""
    E, D = wr.shape
    if h.is_cuda:
        if h.dtype != ACT_DTYPE or wr.dtype != ACT_DTYPE or logits.dtype != torch.float32 or logits.shape[1] != E \
                or not wr.is_contiguous() or logits.stride(0) != E or h.stride(1) != 1 or h.shape[1] < D:
            raise ValueError("router_logits: f16 h / wr, f32 contiguous logits [>= T, E]")
        if zero is not None and (zero.dtype != torch.int32 or not zero.is_contiguous()):
            raise ValueError("router_logits: zero must be contiguous int32")
        _lib.check(_lib.lib().nls_router_logits(h.data_ptr(), h.stride(0), wr.data_ptr(), D, E, logits.data_ptr(), T,
                                                _p(zero), 0 if zero is None else zero.numel(), _stream_ptr(h)),
                   "nls_router_logits")
        return logits
    logits[:T] = h[:T, :D].float() @ wr.float().t()
    if zero is not None:
        zero.zero_()
    return logits


def moe_route(logits: torch.Tensor, T: int, k: int, topw: torch.Tensor, counts: torch.Tensor, xrows: torch.Tensor,
              yrows: torch.Tensor, cap: int, renorm: bool = True, sel: Optional[torch.Tensor] = None,
              counts_zeroed: bool = False):
    """Top-k routing: per-expert row lists (counts / xrows / yrows) and weights topw; `sel` (optional,
    int32 [>= T*k]) receives each (token, slot)'s expert id for device-selected expert launches.
    counts_zeroed: an earlier launch on the stream already zeroed `counts` (router_logits(zero=counts))."""
    E = logits.shape[1]
    if logits.is_cuda:
        if T > 4 and not counts_zeroed:   # one-workgroup launches (T <= 4) zero the counts in-kernel
            counts.zero_()
        _lib.check(_lib.lib().nls_moe_route(logits.data_ptr(), T, E, k, int(renorm), topw.data_ptr(),
                                            counts.data_ptr(), xrows.data_ptr(), yrows.data_ptr(), cap, _p(sel),
                                            _stream_ptr(logits)), "nls_moe_route")
        return
    p = torch.softmax(logits[:T].float(), dim=-1)
    w, e = torch.topk(p, k, dim=-1)
    if renorm:
        w = w / w.sum(dim=-1, keepdim=True)
    topw[:T * k] = w.reshape(-1)
    counts.zero_()
    for t in range(T):
        for j in range(k):
            ex = int(e[t, j])
            c = int(counts[ex])
            xrows[ex * cap + c] = t
            yrows[ex * cap + c] = t * k + j
            counts[ex] += 1
            if sel is not None:
                sel[t * k + j] = ex


def moe_combine_norm(y: torch.Tensor, topw: torch.Tensor, T: int, k: int, resid: torch.Tensor, alpha: float,
                     norm_w: torch.Tensor, eps: float, h: torch.Tensor):
    """moe_combine, then h[:T] = rmsnorm(resid[:T]) * norm_w (the next layer's input norm) in the same launch."""
    if y.is_cuda:
        D = resid.shape[1]
        _lib.check(_lib.lib().nls_moe_combine_norm(y.data_ptr(), topw.data_ptr(), T, k, resid.data_ptr(),
                                                   resid.stride(0), D, float(alpha), norm_w.data_ptr(), float(eps),
                                                   h.data_ptr(), h.stride(0), _stream_ptr(y)), "nls_moe_combine_norm")
        return h
    moe_combine(y, topw, T, k, resid, alpha)
    return rmsnorm(resid, norm_w, h, T, eps)


def moe_combine(y: torch.Tensor, topw: torch.Tensor, T: int, k: int, resid: torch.Tensor, alpha: float = 1.0,
                set_: bool = False):
    """resid[:T] += alpha * sum_j topw[t, j] * y[t*k + j]; set_: resid[:T] = ... (a partial combine from zero)."""
    D = resid.shape[1]
    if y.is_cuda:
        _lib.check(_lib.lib().nls_moe_combine(y.data_ptr(), topw.data_ptr(), T, k, resid.data_ptr(),
                                              resid.stride(0), D, float(alpha), int(set_), _stream_ptr(y)),
                   "nls_moe_combine")
        return
    yy = y[:T * k].float().view(T, k, D)
    c = alpha * (topw[:T * k].view(T, k, 1) * yy).sum(dim=1)
    if set_:
        resid[:T] = c
    else:
        resid[:T] += c
