"""Reference (numpy) codecs for the GGUF block formats the engine executes.

These are the correctness oracles for the HIP dequant-GEMV/GEMM kernels: every
kernel test dequantises the same block bytes here and compares an fp32 matmul.
Block layouts follow ggml's on-disk contract (QK_K = 256):

* Q8_0  {f16 d; i8 qs[32]}                                  34 B / 32 values
* Q4_K  {f16 d; f16 dmin; u8 scales[12]; u8 qs[128]}        144 B / 256
* Q5_K  {f16 d; f16 dmin; u8 scales[12]; u8 qh[32]; u8 qs[128]} 176 B / 256
* Q6_K  {u8 ql[128]; u8 qh[64]; i8 scales[16]; f16 d}       210 B / 256
* Q4_0  {f16 d; u8 qs[16]}                      18 B / 32: x = d*(q - 8)
* Q4_1  {f16 d; f16 m; u8 qs[16]}               20 B / 32: x = d*q + m
* Q5_0  {f16 d; u8 qh[4]; u8 qs[16]}            22 B / 32: x = d*(q - 16)
* Q5_1  {f16 d; f16 m; u8 qh[4]; u8 qs[16]}     24 B / 32: x = d*q + m
  (32-blocks: element j < 16 is the low nibble of qs[j], j >= 16 the high nibble of qs[j-16];
  the 5th bit of element j is bit j of the little-endian u32 qh)
* Q2_K  {u8 scales[16]; u8 qs[64]; f16 d; f16 dmin}          84 B / 256: 16 sub-blocks of 16,
  x = d*(sc & 15)*q - dmin*(sc >> 4), q 2-bit
* Q3_K  {u8 hmask[32]; u8 qs[64]; u8 scales[12]; f16 d}      110 B / 256: 16 sub-blocks of 16,
  x = d*(sc - 32)*(q - 4), q = 2 low bits from qs + 4 * hmask bit, sc 6-bit
  (For both K types, value v of the 128-half n, shift group j, half u, lane l -- v = 128n + 32j + 16u + l
  -- takes bits 2j.. of qs[32n + 16u + l] and, for Q3_K, hmask bit (4n + j) of byte 16u + l.)

The quantisers are simple min/max fits (not llama.cpp's iterative search);
only the *decode* side has to be bit-exact with ggml, because that is what a
GGUF file produced anywhere else contains.
"""
from __future__ import annotations

import numpy as np

from .constants import GGMLType, GGML_BLOCK, QK_K


# ----------------------------------------------------------------------------
# helpers
# ----------------------------------------------------------------------------

def _f16(b: np.ndarray) -> np.ndarray:
    """uint8[..., 2] -> float32[...] (little-endian IEEE half)."""
    return np.ascontiguousarray(b).view(np.float16)[..., 0].astype(np.float32)


def _unpack_k4_scales(sc12: np.ndarray):
    """ggml get_scale_min_k4 for all 8 sub-blocks. sc12: uint8[nb, 12] -> (sc, m) uint8[nb, 8]."""
    q = sc12.astype(np.uint8)
    sc = np.empty(q.shape[:-1] + (8,), np.uint8)
    m = np.empty_like(sc)
    sc[..., :4] = q[..., 0:4] & 63
    m[..., :4] = q[..., 4:8] & 63
    sc[..., 4:] = (q[..., 8:12] & 0xF) | ((q[..., 0:4] >> 6) << 4)
    m[..., 4:] = (q[..., 8:12] >> 4) | ((q[..., 4:8] >> 6) << 4)
    return sc, m


def _pack_k4_scales(sc: np.ndarray, m: np.ndarray) -> np.ndarray:
    """Inverse of _unpack_k4_scales. sc, m: uint8[nb, 8] in [0, 63]."""
    sc = sc.astype(np.uint8)
    m = m.astype(np.uint8)
    q = np.zeros(sc.shape[:-1] + (12,), np.uint8)
    q[..., 0:4] = (sc[..., 0:4] & 63) | ((sc[..., 4:8] >> 4) << 6)
    q[..., 4:8] = (m[..., 0:4] & 63) | ((m[..., 4:8] >> 4) << 6)
    q[..., 8:12] = (sc[..., 4:8] & 0xF) | ((m[..., 4:8] & 0xF) << 4)
    return q


# ----------------------------------------------------------------------------
# dequantisation (bit-exact with ggml)
# ----------------------------------------------------------------------------

def dequant_q8_0(raw: np.ndarray) -> np.ndarray:
    b = raw.reshape(-1, 34)
    d = _f16(b[:, 0:2])
    qs = b[:, 2:34].view(np.int8).astype(np.float32)
    return (d[:, None] * qs).reshape(-1)


def dequant_q4_k(raw: np.ndarray) -> np.ndarray:
    b = raw.reshape(-1, 144)
    d = _f16(b[:, 0:2])
    dmin = _f16(b[:, 2:4])
    sc, m = _unpack_k4_scales(b[:, 4:16])
    qs = b[:, 16:144].reshape(-1, 4, 32)
    lo = (qs & 0xF).astype(np.float32)
    hi = (qs >> 4).astype(np.float32)
    # sub-block 2c -> low nibbles of chunk c; 2c+1 -> high nibbles
    q = np.stack([lo, hi], axis=2).reshape(-1, 8, 32)
    a = (d[:, None] * sc.astype(np.float32))[:, :, None]
    mm = (dmin[:, None] * m.astype(np.float32))[:, :, None]
    return (a * q - mm).reshape(-1)


def dequant_q5_k(raw: np.ndarray) -> np.ndarray:
    b = raw.reshape(-1, 176)
    d = _f16(b[:, 0:2])
    dmin = _f16(b[:, 2:4])
    sc, m = _unpack_k4_scales(b[:, 4:16])
    qh = b[:, 16:48]                       # [nb, 32]
    qs = b[:, 48:176].reshape(-1, 4, 32)
    out = np.empty((b.shape[0], 8, 32), np.float32)
    for c in range(4):
        lo = (qs[:, c] & 0xF) + (((qh >> (2 * c)) & 1) << 4)
        hi = (qs[:, c] >> 4) + (((qh >> (2 * c + 1)) & 1) << 4)
        out[:, 2 * c] = lo
        out[:, 2 * c + 1] = hi
    a = (d[:, None] * sc.astype(np.float32))[:, :, None]
    mm = (dmin[:, None] * m.astype(np.float32))[:, :, None]
    return (a * out - mm).reshape(-1)


def dequant_q6_k(raw: np.ndarray) -> np.ndarray:
    b = raw.reshape(-1, 210)
    ql = b[:, 0:128].astype(np.int32)
    qh = b[:, 128:192].astype(np.int32)
    sc = b[:, 192:208].view(np.int8).astype(np.float32)
    d = _f16(b[:, 208:210])
    out = np.empty((b.shape[0], 256), np.float32)
    for n in range(2):
        l_ = ql[:, 64 * n:64 * n + 64]
        h_ = qh[:, 32 * n:32 * n + 32]
        q1 = ((l_[:, 0:32] & 0xF) | (((h_ >> 0) & 3) << 4)) - 32
        q2 = ((l_[:, 32:64] & 0xF) | (((h_ >> 2) & 3) << 4)) - 32
        q3 = ((l_[:, 0:32] >> 4) | (((h_ >> 4) & 3) << 4)) - 32
        q4 = ((l_[:, 32:64] >> 4) | (((h_ >> 6) & 3) << 4)) - 32
        s = sc[:, 8 * n:8 * n + 8]
        idx = np.arange(32) // 16
        base = 128 * n
        out[:, base + 0:base + 32] = d[:, None] * s[:, idx + 0] * q1
        out[:, base + 32:base + 64] = d[:, None] * s[:, idx + 2] * q2
        out[:, base + 64:base + 96] = d[:, None] * s[:, idx + 4] * q3
        out[:, base + 96:base + 128] = d[:, None] * s[:, idx + 6] * q4
    return out.reshape(-1)


def _q_32(qs: np.ndarray) -> np.ndarray:
    """32-block nibbles: uint8[nb, 16] -> 4-bit values uint8[nb, 32] (j < 16 low nibbles, j >= 16 high)."""
    return np.concatenate([qs & 0xF, qs >> 4], axis=1)


def _qh_32(qh: np.ndarray) -> np.ndarray:
    """uint8[nb, 4] little-endian bit field -> uint8[nb, 32] (bit j of element j)."""
    bits = qh.astype(np.uint32)
    w = bits[:, 0] | (bits[:, 1] << 8) | (bits[:, 2] << 16) | (bits[:, 3] << 24)
    return ((w[:, None] >> np.arange(32, dtype=np.uint32)[None, :]) & 1).astype(np.uint8)


def unpack_q5_1_family(raw: np.ndarray, ggml_type: int):
    """Q4_0 / Q4_1 / Q5_0 / Q5_1 blocks -> (d f32[nb], m f32[nb], q uint8[nb, 32]) with x = d*q + m EXACTLY
    (m = -8d / -16d for the symmetric types: a power-of-two multiple of an f16, exact in f16 too)."""
    t = GGMLType(ggml_type)
    nbytes = GGML_BLOCK[t][1]
    b = np.ascontiguousarray(raw).view(np.uint8).reshape(-1, nbytes)
    d = _f16(b[:, 0:2])
    if t == GGMLType.Q4_0:
        return d, -8.0 * d, _q_32(b[:, 2:18])
    if t == GGMLType.Q4_1:
        return d, _f16(b[:, 2:4]), _q_32(b[:, 4:20])
    if t == GGMLType.Q5_0:
        return d, -16.0 * d, _q_32(b[:, 6:22]) | (_qh_32(b[:, 2:6]) << 4)
    if t == GGMLType.Q5_1:
        return d, _f16(b[:, 2:4]), _q_32(b[:, 8:24]) | (_qh_32(b[:, 4:8]) << 4)
    raise ValueError(t.name)


def _k_lowbit_index():
    """For the 2-bit K layouts: value v -> (qs byte, shift); v = 128n + 32j + 16u + l."""
    v = np.arange(256)
    n, j, u, l = v // 128, (v // 32) % 4, (v // 16) % 2, v % 16
    return 32 * n + 16 * u + l, 2 * j, 4 * n + j, 16 * u + l


_KIDX = _k_lowbit_index()


def unpack_q2_k(raw: np.ndarray):
    """-> (a f32[nb, 16], c f32[nb, 16], q uint8[nb, 256]): x = a[v // 16] * q[v] + c[v // 16]."""
    b = np.ascontiguousarray(raw).view(np.uint8).reshape(-1, 84)
    sc = b[:, 0:16]
    qs = b[:, 16:80]
    d = _f16(b[:, 80:82])
    dmin = _f16(b[:, 82:84])
    byte, shift, _, _ = _KIDX
    q = (qs[:, byte] >> shift[None, :]) & 3
    return d[:, None] * (sc & 0xF).astype(np.float32), -dmin[:, None] * (sc >> 4).astype(np.float32), q


def _unpack_q3_scales(sc12: np.ndarray) -> np.ndarray:
    """ggml Q3_K 6-bit scales (kmask1/kmask2 shuffle): uint8[nb, 12] -> int[nb, 16] in [0, 63]."""
    a = sc12.astype(np.uint32)
    aux = [a[:, 4 * i] | (a[:, 4 * i + 1] << 8) | (a[:, 4 * i + 2] << 16) | (a[:, 4 * i + 3] << 24) for i in range(3)]
    k1, k2 = 0x03030303, 0x0F0F0F0F
    tmp = aux[2]
    w = [(aux[0] & k2) | (((tmp >> 0) & k1) << 4), (aux[1] & k2) | (((tmp >> 2) & k1) << 4),
         ((aux[0] >> 4) & k2) | (((tmp >> 4) & k1) << 4), ((aux[1] >> 4) & k2) | (((tmp >> 6) & k1) << 4)]
    out = np.empty((sc12.shape[0], 16), np.int32)
    for i in range(4):
        for k in range(4):
            out[:, 4 * i + k] = (w[i] >> (8 * k)) & 0xFF
    return out


def _pack_q3_scales(s: np.ndarray) -> np.ndarray:
    """Inverse of _unpack_q3_scales: int[nb, 16] in [0, 63] -> uint8[nb, 12]."""
    s = s.astype(np.uint32)
    out = np.zeros((s.shape[0], 12), np.uint8)
    for i in range(16):
        lo, hi = s[:, i] & 0xF, s[:, i] >> 4
        if i < 8:
            out[:, i] |= lo.astype(np.uint8)
        else:
            out[:, i - 8] |= (lo << 4).astype(np.uint8)
        out[:, 8 + (i % 4)] |= (hi << (2 * (i // 4))).astype(np.uint8)
    return out


def unpack_q3_k(raw: np.ndarray):
    """-> (d f32[nb], s int[nb, 16] (signed, sc - 32), q3 uint8[nb, 256] in [0, 7]): x = d*s*(q3 - 4)."""
    b = np.ascontiguousarray(raw).view(np.uint8).reshape(-1, 110)
    hm = b[:, 0:32]
    qs = b[:, 32:96]
    s = _unpack_q3_scales(b[:, 96:108]) - 32
    d = _f16(b[:, 108:110])
    byte, shift, hbit, hbyte = _KIDX
    q = ((qs[:, byte] >> shift[None, :]) & 3) | (((hm[:, hbyte] >> hbit[None, :]) & 1) << 2)
    return d, s, q.astype(np.uint8)


def dequantize(raw: np.ndarray, ggml_type: int, shape) -> np.ndarray:
    """Dequantise raw tensor bytes to float32 with numpy shape `shape` (row-major, innermost last)."""
    t = GGMLType(ggml_type)
    raw = np.ascontiguousarray(raw).view(np.uint8).reshape(-1)
    if t == GGMLType.F32:
        out = raw.view(np.float32).astype(np.float32)
    elif t == GGMLType.F16:
        out = raw.view(np.float16).astype(np.float32)
    elif t == GGMLType.BF16:
        out = (raw.view(np.uint16).astype(np.uint32) << 16).view(np.float32)
    elif t == GGMLType.Q8_0:
        out = dequant_q8_0(raw)
    elif t == GGMLType.Q4_K:
        out = dequant_q4_k(raw)
    elif t == GGMLType.Q5_K:
        out = dequant_q5_k(raw)
    elif t == GGMLType.Q6_K:
        out = dequant_q6_k(raw)
    elif t in (GGMLType.Q4_0, GGMLType.Q4_1, GGMLType.Q5_0, GGMLType.Q5_1):
        d, m, q = unpack_q5_1_family(raw, t)
        out = (d[:, None] * q.astype(np.float32) + m[:, None]).reshape(-1)
    elif t == GGMLType.Q2_K:
        a, c, q = unpack_q2_k(raw)
        out = (np.repeat(a, 16, axis=1) * q.astype(np.float32) + np.repeat(c, 16, axis=1)).reshape(-1)
    elif t == GGMLType.Q3_K:
        d, sc, q = unpack_q3_k(raw)
        out = (d[:, None] * np.repeat(sc.astype(np.float32), 16, axis=1) * (q.astype(np.float32) - 4)).reshape(-1)
    else:
        raise NotImplementedError(f"dequantize: {t.name}")
    return out.reshape(shape)


# ----------------------------------------------------------------------------
# quantisation (simple min/max fits; decode-compatible with ggml)
# ----------------------------------------------------------------------------

def _to_f16_bytes(x: np.ndarray) -> np.ndarray:
    return x.astype(np.float16).view(np.uint8).reshape(x.shape + (2,))


def quant_q8_0(x: np.ndarray) -> np.ndarray:
    x = x.reshape(-1, 32).astype(np.float32)
    amax = np.abs(x).max(axis=1)
    d = (amax / 127.0).astype(np.float16).astype(np.float32)
    inv = np.where(d > 0, 1.0 / np.where(d > 0, d, 1), 0)
    q = np.clip(np.rint(x * inv[:, None]), -127, 127).astype(np.int8)
    out = np.empty((x.shape[0], 34), np.uint8)
    out[:, 0:2] = _to_f16_bytes(d)
    out[:, 2:] = q.view(np.uint8)
    return out.reshape(-1)


def _fit_k4(x: np.ndarray, qmax: int):
    """Per 32-sub-block affine fit x ~ d*sc*q - dmin*m (q in [0,qmax]). x: [nb, 8, 32]."""
    mn = np.minimum(x.min(axis=2), 0.0)
    mx = x.max(axis=2)
    scale = (mx - mn) / qmax
    mins = -mn
    d = (scale.max(axis=1) / 63.0).astype(np.float16).astype(np.float32)
    dmin = (mins.max(axis=1) / 63.0).astype(np.float16).astype(np.float32)
    sc = np.clip(np.rint(scale / np.where(d > 0, d, 1)[:, None]), 0, 63).astype(np.uint8)
    m = np.clip(np.rint(mins / np.where(dmin > 0, dmin, 1)[:, None]), 0, 63).astype(np.uint8)
    a = d[:, None] * sc
    b = dmin[:, None] * m
    q = np.rint((x + b[:, :, None]) / np.where(a > 0, a, 1)[:, :, None])
    q = np.clip(q, 0, qmax).astype(np.uint8)
    return d, dmin, sc, m, q


def quant_q4_k(x: np.ndarray) -> np.ndarray:
    x = x.reshape(-1, 8, 32).astype(np.float32)
    d, dmin, sc, m, q = _fit_k4(x, 15)
    nb = x.shape[0]
    out = np.empty((nb, 144), np.uint8)
    out[:, 0:2] = _to_f16_bytes(d)
    out[:, 2:4] = _to_f16_bytes(dmin)
    out[:, 4:16] = _pack_k4_scales(sc, m)
    q = q.reshape(nb, 4, 2, 32)
    out[:, 16:144] = (q[:, :, 0] | (q[:, :, 1] << 4)).reshape(nb, 128)
    return out.reshape(-1)


def quant_q5_k(x: np.ndarray) -> np.ndarray:
    x = x.reshape(-1, 8, 32).astype(np.float32)
    d, dmin, sc, m, q = _fit_k4(x, 31)
    nb = x.shape[0]
    out = np.zeros((nb, 176), np.uint8)
    out[:, 0:2] = _to_f16_bytes(d)
    out[:, 2:4] = _to_f16_bytes(dmin)
    out[:, 4:16] = _pack_k4_scales(sc, m)
    q = q.reshape(nb, 4, 2, 32)
    qh = np.zeros((nb, 32), np.uint8)
    for c in range(4):
        qh |= ((q[:, c, 0] >> 4) & 1) << (2 * c)
        qh |= ((q[:, c, 1] >> 4) & 1) << (2 * c + 1)
    out[:, 16:48] = qh
    out[:, 48:176] = ((q[:, :, 0] & 0xF) | ((q[:, :, 1] & 0xF) << 4)).reshape(nb, 128)
    return out.reshape(-1)


def quant_q6_k(x: np.ndarray) -> np.ndarray:
    x = x.reshape(-1, 16, 16).astype(np.float32)      # 16 sub-blocks of 16
    nb = x.shape[0]
    amax = np.abs(x).max(axis=2)
    scale = amax / 31.0
    d = (np.abs(scale).max(axis=1) / 127.0).astype(np.float16).astype(np.float32)
    sc = np.clip(np.rint(scale / np.where(d > 0, d, 1)[:, None]), -128, 127).astype(np.int8)
    a = d[:, None] * sc.astype(np.float32)
    q = np.clip(np.rint(x / np.where(a != 0, a, 1)[:, :, None]), -32, 31).astype(np.int32) + 32
    q = q.reshape(nb, 256)
    out = np.empty((nb, 210), np.uint8)
    ql = np.zeros((nb, 128), np.uint8)
    qh = np.zeros((nb, 64), np.uint8)
    for n in range(2):
        v = q[:, 128 * n:128 * n + 128]
        q1, q2, q3, q4 = v[:, 0:32], v[:, 32:64], v[:, 64:96], v[:, 96:128]
        ql[:, 64 * n:64 * n + 32] = ((q1 & 0xF) | ((q3 & 0xF) << 4)).astype(np.uint8)
        ql[:, 64 * n + 32:64 * n + 64] = ((q2 & 0xF) | ((q4 & 0xF) << 4)).astype(np.uint8)
        qh[:, 32 * n:32 * n + 32] = ((q1 >> 4) | ((q2 >> 4) << 2) | ((q3 >> 4) << 4) | ((q4 >> 4) << 6)).astype(np.uint8)
    out[:, 0:128] = ql
    out[:, 128:192] = qh
    out[:, 192:208] = sc.view(np.uint8)
    out[:, 208:210] = _to_f16_bytes(d)
    return out.reshape(-1)


def _pack_32(q: np.ndarray) -> np.ndarray:
    """4-bit values uint8[nb, 32] -> 32-block nibbles uint8[nb, 16]."""
    return ((q[:, :16] & 0xF) | ((q[:, 16:] & 0xF) << 4)).astype(np.uint8)


def _pack_qh_32(q: np.ndarray) -> np.ndarray:
    w = (((q.astype(np.uint32) >> 4) & 1) << np.arange(32, dtype=np.uint32)[None, :]).sum(axis=1).astype(np.uint32)
    return w.view(np.uint8).reshape(-1, 4)


def quant_q5_1_family(x: np.ndarray, ggml_type: int) -> np.ndarray:
    """Q4_0 / Q4_1 / Q5_0 / Q5_1 by per-block min/max (symmetric types: amax)."""
    t = GGMLType(ggml_type)
    x = x.reshape(-1, 32).astype(np.float32)
    nb = x.shape[0]
    bits = 5 if t in (GGMLType.Q5_0, GGMLType.Q5_1) else 4
    qmax = (1 << bits) - 1
    if t in (GGMLType.Q4_0, GGMLType.Q5_0):
        half = 1 << (bits - 1)
        amax_i = np.abs(x).argmax(axis=1)
        mx = x[np.arange(nb), amax_i]
        d = (mx / -half).astype(np.float16).astype(np.float32)
        inv = np.where(d != 0, 1.0 / np.where(d != 0, d, 1), 0)
        q = np.clip(np.rint(x * inv[:, None]) + half, 0, qmax).astype(np.uint8)
        m = None
    else:
        mn, mxv = x.min(axis=1), x.max(axis=1)
        d = ((mxv - mn) / qmax).astype(np.float16).astype(np.float32)
        m = mn.astype(np.float16).astype(np.float32)
        inv = np.where(d > 0, 1.0 / np.where(d > 0, d, 1), 0)
        q = np.clip(np.rint((x - m[:, None]) * inv[:, None]), 0, qmax).astype(np.uint8)
    out = [_to_f16_bytes(d)]
    if m is not None:
        out.append(_to_f16_bytes(m))
    if bits == 5:
        out.append(_pack_qh_32(q))
    out.append(_pack_32(q))
    return np.concatenate(out, axis=1).reshape(-1)


def quant_q2_k(x: np.ndarray) -> np.ndarray:
    x = x.reshape(-1, 16, 16).astype(np.float32)
    nb = x.shape[0]
    mn = np.minimum(x.min(axis=2), 0.0)
    scale = (x.max(axis=2) - mn) / 3.0
    d = (scale.max(axis=1) / 15.0).astype(np.float16).astype(np.float32)
    dmin = ((-mn).max(axis=1) / 15.0).astype(np.float16).astype(np.float32)
    sc = np.clip(np.rint(scale / np.where(d > 0, d, 1)[:, None]), 0, 15).astype(np.uint8)
    m = np.clip(np.rint(-mn / np.where(dmin > 0, dmin, 1)[:, None]), 0, 15).astype(np.uint8)
    a = d[:, None] * sc
    q = np.clip(np.rint((x + (dmin[:, None] * m)[:, :, None]) / np.where(a > 0, a, 1)[:, :, None]), 0, 3)
    q = q.reshape(nb, 256).astype(np.uint8)
    byte, shift, _, _ = _KIDX
    qs = np.zeros((nb, 64), np.uint8)
    for v in range(256):
        qs[:, byte[v]] |= (q[:, v] << shift[v]).astype(np.uint8)
    out = np.empty((nb, 84), np.uint8)
    out[:, 0:16] = sc | (m << 4)
    out[:, 16:80] = qs
    out[:, 80:82] = _to_f16_bytes(d)
    out[:, 82:84] = _to_f16_bytes(dmin)
    return out.reshape(-1)


def quant_q3_k(x: np.ndarray) -> np.ndarray:
    x = x.reshape(-1, 16, 16).astype(np.float32)
    nb = x.shape[0]
    scale = np.abs(x).max(axis=2) / 4.0
    d = (scale.max(axis=1) / 31.0).astype(np.float16).astype(np.float32)
    s = np.clip(np.rint(scale / np.where(d > 0, d, 1)[:, None]), -32, 31).astype(np.int32)
    a = d[:, None] * s
    q = np.clip(np.rint(x / np.where(a != 0, a, 1)[:, :, None]) + 4, 0, 7).astype(np.uint8).reshape(nb, 256)
    byte, shift, hbit, hbyte = _KIDX
    qs = np.zeros((nb, 64), np.uint8)
    hm = np.zeros((nb, 32), np.uint8)
    for v in range(256):
        qs[:, byte[v]] |= ((q[:, v] & 3) << shift[v]).astype(np.uint8)
        hm[:, hbyte[v]] |= (((q[:, v] >> 2) & 1) << hbit[v]).astype(np.uint8)
    out = np.empty((nb, 110), np.uint8)
    out[:, 0:32] = hm
    out[:, 32:96] = qs
    out[:, 96:108] = _pack_q3_scales(s + 32)
    out[:, 108:110] = _to_f16_bytes(d)
    return out.reshape(-1)


def quantize(x: np.ndarray, ggml_type: int) -> np.ndarray:
    """float array -> raw uint8 bytes in the given ggml type (row-major)."""
    t = GGMLType(ggml_type)
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    if t == GGMLType.F32:
        return x.view(np.uint8).copy()
    if t == GGMLType.F16:
        return x.astype(np.float16).view(np.uint8).copy()
    if t == GGMLType.BF16:
        u = x.view(np.uint32)
        r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
        return r.view(np.uint8).copy()
    if t == GGMLType.Q8_0:
        return quant_q8_0(x)
    if t == GGMLType.Q4_K:
        return quant_q4_k(x)
    if t == GGMLType.Q5_K:
        return quant_q5_k(x)
    if t == GGMLType.Q6_K:
        return quant_q6_k(x)
    if t in (GGMLType.Q4_0, GGMLType.Q4_1, GGMLType.Q5_0, GGMLType.Q5_1):
        return quant_q5_1_family(x, t)
    if t == GGMLType.Q2_K:
        return quant_q2_k(x)
    if t == GGMLType.Q3_K:
        return quant_q3_k(x)
    raise NotImplementedError(f"quantize: {t.name}")


# ----------------------------------------------------------------------------
# random-init blocks (fast path for multi-GB synthetic checkpoints)
# ----------------------------------------------------------------------------

def random_blocks(ggml_type: int, n_elements: int, std: float, rng: np.random.Generator) -> np.ndarray:
    """Random but well-formed block bytes whose dequantised values have roughly
    zero mean and standard deviation `std`. Generating block bytes directly
    (instead of quantising float weights) makes an 8B/70B random checkpoint a
    few seconds of numpy instead of minutes."""
    t = GGMLType(ggml_type)
    blk, nbytes = GGML_BLOCK[t]
    nb = n_elements // blk
    if t in (GGMLType.F32, GGMLType.F16, GGMLType.BF16):
        x = rng.standard_normal(n_elements, dtype=np.float32) * std
        return quantize(x, t)
    raw = rng.integers(0, 256, size=(nb, nbytes), dtype=np.uint8)
    if t == GGMLType.Q8_0:
        # uniform int8 std ~ 73.6
        d = np.full(nb, std / 73.6, np.float32)
        raw[:, 0:2] = _to_f16_bytes(d)
        return raw.reshape(-1)
    if t in (GGMLType.Q4_K, GGMLType.Q5_K):
        qmax = 15 if t == GGMLType.Q4_K else 31
        sc = rng.integers(24, 41, size=(nb, 8)).astype(np.uint8)
        q_std = np.sqrt((qmax + 1) ** 2 - 1) / np.sqrt(12.0)
        d = np.full(nb, std / (32.0 * q_std), np.float32)
        # centre: dmin*m ~ d*sc*qmax/2 ; pick dmin = d*qmax/2*... so m fits in 6 bits
        dmin = d * (qmax / 2.0) * 40.0 / 60.0
        m = np.clip(np.rint(d[:, None] * sc * (qmax / 2.0) / dmin[:, None]), 0, 63).astype(np.uint8)
        raw[:, 0:2] = _to_f16_bytes(d)
        raw[:, 2:4] = _to_f16_bytes(dmin)
        raw[:, 4:16] = _pack_k4_scales(sc, m)
        return raw.reshape(-1)
    if t == GGMLType.Q6_K:
        sc = rng.integers(24, 41, size=(nb, 16)).astype(np.int8)
        q_std = np.sqrt(64 ** 2 - 1) / np.sqrt(12.0)
        d = np.full(nb, std / (32.0 * q_std), np.float32)
        raw[:, 192:208] = sc.view(np.uint8)
        raw[:, 208:210] = _to_f16_bytes(d)
        return raw.reshape(-1)
    if t in (GGMLType.Q4_0, GGMLType.Q4_1, GGMLType.Q5_0, GGMLType.Q5_1):
        qmax = 31 if t in (GGMLType.Q5_0, GGMLType.Q5_1) else 15
        q_std = np.sqrt((qmax + 1) ** 2 - 1) / np.sqrt(12.0)
        d = np.full(nb, std / q_std, np.float32) * rng.uniform(0.8, 1.2, nb).astype(np.float32)
        raw[:, 0:2] = _to_f16_bytes(d)
        if t in (GGMLType.Q4_1, GGMLType.Q5_1):      # zero-mean: m = -d * qmax / 2
            raw[:, 2:4] = _to_f16_bytes(-d * qmax / 2.0)
        return raw.reshape(-1)
    if t == GGMLType.Q2_K:
        sc = rng.integers(6, 12, size=(nb, 16)).astype(np.uint8)
        q_std = np.sqrt(4 ** 2 - 1) / np.sqrt(12.0)
        d = np.full(nb, std / (9.0 * q_std), np.float32)
        dmin = d * 1.5 * 9.0 / 8.0
        m = np.clip(np.rint(d[:, None] * sc * 1.5 / dmin[:, None]), 0, 15).astype(np.uint8)
        raw[:, 0:16] = sc | (m << 4)
        raw[:, 80:82] = _to_f16_bytes(d)
        raw[:, 82:84] = _to_f16_bytes(dmin)
        return raw.reshape(-1)
    if t == GGMLType.Q3_K:
        s = rng.integers(40, 56, size=(nb, 16))                  # sc - 32 in [8, 24)
        q_std = np.sqrt(8 ** 2 - 1) / np.sqrt(12.0)
        d = np.full(nb, std / (16.0 * q_std), np.float32)
        raw[:, 96:108] = _pack_q3_scales(s)
        raw[:, 108:110] = _to_f16_bytes(d)
        return raw.reshape(-1)
    raise NotImplementedError(f"random_blocks: {t.name}")


__all__ = ["dequantize", "quantize", "random_blocks", "QK_K"]
