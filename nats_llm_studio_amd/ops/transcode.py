"""Load-time re-encoding of the GGUF block formats that have no kernels of their own into formats that
do -- losslessly wherever the value set allows it (torch ops on the raw bytes, on the load device):

  Q4_0 / Q4_1 / Q5_0 / Q5_1  -> device type Q51 (csrc/kernels/common.h QT_Q51): per 32-value block
                                 x = d*q + m with q 5-bit; the symmetric types take m = -8d / -16d,
                                 a power-of-two multiple of an f16, so EVERY value is reproduced exactly.
                                 Same bytes as Q5_1 (1.33x a Q4_0 block), Q5_K's tile arrangement.
  Q3_K                        -> Q6_K, exactly: x = d*(sc-32)*(q3-4) with q3 in [0, 7] is
                                 d6*sc6*(q6-32) with d6 = d, sc6 = sc-32 (int8), q6 = q3 + 28.
  Q2_K                        -> F16 (x = d*sc*q - dmin*m rounded once to f16; no K-quant with
                                 16-value sub-blocks AND a min offset exists on the device).
Embedding tables ("rows" layout, gathered): Q4_0 / Q5_0 -> Q8_0 rows (exact), Q3_K -> Q6_K rows,
the affine types -> F16 rows.

`pull_model` (the reference's `lms get <any id>`, /root/reference/nats_llm_studio.go:46-59) can
therefore materialise any of these GGUF mixes and `chat_model` serves it; the CPU reference path keeps
decoding the ORIGINAL bytes with gguf/quants.py (the oracle of the tests).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch

from ..gguf.constants import GGMLType, GGML_BLOCK
from ..gguf.quants import _KIDX

QT_Q51 = 101
AFFINE32 = (GGMLType.Q4_0, GGMLType.Q4_1, GGMLType.Q5_0, GGMLType.Q5_1)
TRANSCODED = AFFINE32 + (GGMLType.Q2_K, GGMLType.Q3_K)


def _f16(b: torch.Tensor) -> torch.Tensor:
    """uint8 [..., 2] -> float16 [...]."""
    return b.contiguous().view(torch.float16).squeeze(-1)


def _bits32(qh: torch.Tensor) -> torch.Tensor:
    """uint8 [nb, 4] little-endian -> uint8 [nb, 32] (bit j of element j)."""
    w = qh.to(torch.int64)
    w = w[:, 0] | (w[:, 1] << 8) | (w[:, 2] << 16) | (w[:, 3] << 24)
    return ((w[:, None] >> torch.arange(32, device=qh.device)[None, :]) & 1).to(torch.uint8)


def unpack_affine32(raw: torch.Tensor, t: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Q4_0/Q4_1/Q5_0/Q5_1 bytes -> (d f16 [nb], m f16 [nb], q uint8 [nb, 32]), x = d*q + m exactly."""
    t = GGMLType(t)
    b = raw.reshape(-1, GGML_BLOCK[t][1])
    d = _f16(b[:, 0:2])
    if t in (GGMLType.Q4_0, GGMLType.Q5_0):
        m = (d.float() * (-8.0 if t == GGMLType.Q4_0 else -16.0)).to(torch.float16)   # exact (x 2^k)
        qo = 2 if t == GGMLType.Q4_0 else 6
    else:
        m = _f16(b[:, 2:4])
        qo = 4 if t == GGMLType.Q4_1 else 8
    qs = b[:, qo:qo + 16]
    q = torch.cat([qs & 0xF, qs >> 4], dim=1)
    if t in (GGMLType.Q5_0, GGMLType.Q5_1):
        ho = 2 if t == GGMLType.Q5_0 else 4
        q = q | (_bits32(b[:, ho:ho + 4]) << 4)
    return d, m, q


def q51_tiled(raw: torch.Tensor, t: int, rows: int, K: int) -> torch.Tensor:
    """Tiled Q51 layout (common.h): per (16-row tile, 256-value super-block) 3072 B =
    [16 rows x (8 f16 d | 8 f16 m)] | QH[g][r][8] | P_h[g][r] -- the last two exactly as Q5_K's, so the
    32-blocks t = 0..7 of a super-block are re-packed the way Q5_K stores its sub-blocks (low / high
    nibbles of chunk t >> 1, 5th bit = bit t of qh)."""
    nb = K // 256
    d, m, q = unpack_affine32(raw, t)
    d = d.reshape(rows, nb, 8)
    m = m.reshape(rows, nb, 8)
    q = q.reshape(rows, nb, 8, 32)
    sc = torch.cat([d.contiguous().view(torch.uint8).reshape(rows, nb, 16),
                    m.contiguous().view(torch.uint8).reshape(rows, nb, 16)], dim=2)
    qs = ((q[:, :, 0::2] & 0xF) | ((q[:, :, 1::2] & 0xF) << 4)).reshape(rows, nb, 128)
    sh = torch.arange(8, device=q.device, dtype=torch.int32).view(1, 1, 8, 1)
    qh = (((q.to(torch.int32) >> 4) & 1) << sh).sum(dim=2).to(torch.uint8)          # [rows, nb, 32]
    vb = torch.cat([sc, qh, qs], dim=2)                                              # [rows, nb, 192]
    rp = (rows + 15) // 16 * 16
    if rp != rows:
        vb = torch.cat([vb, torch.zeros(rp - rows, nb, 192, dtype=torch.uint8, device=vb.device)])
    T = rp // 16
    B = vb.reshape(T, 16, nb, 192)
    parts = [B[..., 0:32].permute(0, 2, 1, 3).reshape(T, nb, 512),
             B[..., 32:64].reshape(T, 16, nb, 4, 8).permute(0, 2, 3, 1, 4).reshape(T, nb, 512),
             B[..., 64:192].reshape(T, 16, nb, 2, 2, 4, 8).permute(0, 2, 3, 5, 1, 4, 6).reshape(T, nb, 2048)]
    return torch.cat(parts, dim=2).reshape(-1).contiguous()


_IDX = {}


def _kidx(dev):
    if dev not in _IDX:
        _IDX[dev] = tuple(torch.from_numpy(np.asarray(a)).to(dev) for a in _KIDX)
    return _IDX[dev]


def q3k_to_q6k(raw: torch.Tensor) -> torch.Tensor:
    """Q3_K blocks (110 B) -> Q6_K blocks (210 B) with identical values."""
    b = raw.reshape(-1, 110)
    nb = b.shape[0]
    hm, qs, scb, dbytes = b[:, 0:32], b[:, 32:96], b[:, 96:108].to(torch.int32), b[:, 108:110]
    j = torch.arange(16, device=b.device)
    lo_src = torch.where(j < 8, j, j - 8)
    lo = torch.where(j < 8, scb[:, lo_src] & 0xF, scb[:, lo_src] >> 4)
    hi = (scb[:, 8 + j % 4] >> (2 * (j // 4))) & 3
    s6 = ((lo | (hi << 4)) - 32).to(torch.int8)
    byte, shift, hbit, hbyte = _kidx(b.device)
    q3 = ((qs[:, byte].to(torch.int32) >> shift) & 3) | (((hm[:, hbyte].to(torch.int32) >> hbit) & 1) << 2)
    q6 = q3 + 28                                                                       # [nb, 256] in [28, 35]
    ql = torch.empty(nb, 128, dtype=torch.int32, device=b.device)
    qh = torch.empty(nb, 64, dtype=torch.int32, device=b.device)
    for n in range(2):
        v = q6[:, 128 * n:128 * n + 128]
        q1, q2, q3_, q4 = v[:, 0:32], v[:, 32:64], v[:, 64:96], v[:, 96:128]
        ql[:, 64 * n:64 * n + 32] = (q1 & 0xF) | ((q3_ & 0xF) << 4)
        ql[:, 64 * n + 32:64 * n + 64] = (q2 & 0xF) | ((q4 & 0xF) << 4)
        qh[:, 32 * n:32 * n + 32] = (q1 >> 4) | ((q2 >> 4) << 2) | ((q3_ >> 4) << 4) | ((q4 >> 4) << 6)
    out = torch.cat([ql.to(torch.uint8), qh.to(torch.uint8), s6.view(torch.uint8), dbytes], dim=1)
    return out.reshape(-1).contiguous()


def dequant_f16(raw: torch.Tensor, t: int) -> torch.Tensor:
    """Q2_K or an affine 32-block type -> f16 values (flat), computed in fp32 and rounded once."""
    t = GGMLType(t)
    if t in AFFINE32:
        d, m, q = unpack_affine32(raw, t)
        return (d.float()[:, None] * q.float() + m.float()[:, None]).to(torch.float16).reshape(-1)
    if t == GGMLType.Q2_K:
        b = raw.reshape(-1, 84)
        sc = b[:, 0:16].to(torch.int32)
        qs = b[:, 16:80].to(torch.int32)
        d, dmin = _f16(b[:, 80:82]).float(), _f16(b[:, 82:84]).float()
        byte, shift, _, _ = _kidx(b.device)
        q = ((qs[:, byte] >> shift) & 3).float()
        a = (d[:, None] * (sc & 0xF).float()).repeat_interleave(16, dim=1)
        c = (-dmin[:, None] * (sc >> 4).float()).repeat_interleave(16, dim=1)
        return (a * q + c).to(torch.float16).reshape(-1)
    raise ValueError(t.name)


def affine32_to_q8_0(raw: torch.Tensor, t: int) -> torch.Tensor:
    """Q4_0 / Q5_0 (symmetric) -> Q8_0 blocks, exactly (qs = q - 8 / q - 16, same d)."""
    t = GGMLType(t)
    b = raw.reshape(-1, GGML_BLOCK[t][1])
    _, _, q = unpack_affine32(raw, t)
    qs = (q.to(torch.int16) - (8 if t == GGMLType.Q4_0 else 16)).to(torch.int8).view(torch.uint8)
    return torch.cat([b[:, 0:2], qs], dim=1).reshape(-1).contiguous()


def device_form(raw: torch.Tensor, ggml_type: int, rows: int, K: int, layout: str):
    """(uint8 bytes, device type) a transcoded format runs as; `raw` already on the load device. For the
    "tiled" layout the bytes are final (tile layout applied); for "rows" they are ggml-format bytes of the
    device type (ops.to_device_layout still applies)."""
    t = GGMLType(ggml_type)
    if layout == "tiled":
        if t in AFFINE32:
            return q51_tiled(raw, t, rows, K), QT_Q51
        if t == GGMLType.Q3_K:
            return q3k_to_q6k(raw), int(GGMLType.Q6_K)
        return dequant_f16(raw, t).view(torch.uint8), int(GGMLType.F16)
    if t in (GGMLType.Q4_0, GGMLType.Q5_0):
        return affine32_to_q8_0(raw, t), int(GGMLType.Q8_0)
    if t == GGMLType.Q3_K:
        return q3k_to_q6k(raw), int(GGMLType.Q6_K)
    return dequant_f16(raw, t).view(torch.uint8), int(GGMLType.F16)
