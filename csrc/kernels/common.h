// Shared device helpers for the gfx950 (CDNA4) kernels of nats_llm_studio_amd.
//
// Weight formats live on the device in GGUF block encodings (never pre-dequantised:
// decode is HBM-bound), re-tiled at load time ("tiled" layout, same bytes):
//   rows are padded to 16 and grouped into 16-row tiles; for every (tile, 256-value
//   super-block) the 16 rows' blocks form ONE contiguous "tile-block" of TB bytes,
//   arranged so that each wave-wide 16-B load instruction of the GEMV reads 1 KiB
//   contiguous (lane l = 16*g + r -> byte 16*l of a 1 KiB piece). Tile-blocks are
//   ordered [tile][super-block], so a wave walking K streams sequential memory.
//     Q4_K  TB=2304: hdr[r] (16) | P0[g][r] (16) | P1[g][r] (16)       (P = qs pieces g, g+4)
//     Q5_K  TB=2816: hdr[r] | qh[h][r] (16, h=g&1) | P0[g][r] | P1[g][r]
//     Q6_K  TB=3360: qa[l] | qb[l] | qh[l] (16 each) | sc[r] (16) | d[r] (2)
//     Q8_0  TB=4352: qs[i][l] (4 x 16) | d[r][8] (f16)
//     F16/BF16 TB=8192: v[t][l] (8 x 16);  F32 TB=16384: v[t][l] (16 x 16)
// Embedding tables keep a row-major "rows" layout (gathered, not streamed):
//   Q4_K/Q5_K native blocks; Q6_K planes ql|qh|sc|d; Q8_0 planes qs|d.
//
// MFMA operand mapping (v_mfma_f32_16x16x32_bf16): lane l = 16*g + r holds
// A[row r][k = 8g + j] and B[k = 8g + j][col r], j = 0..7. The contraction order
// inside K is free, so each format picks, per 256-value super-block, a lane->k
// assignment where (a) a lane's weight bytes are contiguous 16-B loads and (b)
// each K-step's 8 values are 8 *consecutive* k (so the activation fragment is one
// 16-B load). xoff(t, g) below is the first k of K-step t for lane group g.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

enum QType : int {
  QT_F32 = 0, QT_F16 = 1, QT_Q8_0 = 8, QT_Q4_K = 12, QT_Q5_K = 13, QT_Q6_K = 14, QT_BF16 = 30
};

#define DEVI __device__ __forceinline__

DEVI float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
DEVI float bf2f(uint16_t b) { return __builtin_bit_cast(float, ((uint32_t)b) << 16); }
DEVI uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

DEVI u32x4 ld16(const void* p) { return *reinterpret_cast<const u32x4*>(p); }
DEVI u32x4 ld16_nt(const void* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

// ggml get_scale_min_k4 over the 12 packed scale bytes held as 3 dwords.
// HI selects the j >= 4 branch at compile time (the sub-block index itself may be
// lane-dependent, the branch never is for the lane->k maps used here).
DEVI int byte_of(uint32_t s0, uint32_t s1, uint32_t s2, int i) {
  uint32_t w = i < 4 ? s0 : (i < 8 ? s1 : s2);
  return (w >> (8 * (i & 3))) & 0xFF;
}
template <bool HI>
DEVI void k4_scale_min_t(int j, uint32_t s0, uint32_t s1, uint32_t s2, int& sc, int& m) {
  if constexpr (!HI) {
    sc = byte_of(s0, s1, s2, j) & 63;
    m = byte_of(s0, s1, s2, j + 4) & 63;
  } else {
    const int b4 = byte_of(s0, s1, s2, j + 4);
    sc = (b4 & 0xF) | ((byte_of(s0, s1, s2, j - 4) >> 6) << 4);
    m = (b4 >> 4) | ((byte_of(s0, s1, s2, j) >> 6) << 4);
  }
}
DEVI void k4_scale_min(int j, uint32_t s0, uint32_t s1, uint32_t s2, int& sc, int& m) {
  if (j < 4) k4_scale_min_t<false>(j, s0, s1, s2, sc, m);
  else k4_scale_min_t<true>(j, s0, s1, s2, sc, m);
}

DEVI bf16x8 pack8(const float* v) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[j];
  return r;
}

// ---------------------------------------------------------------------------
// Per-format raw loads (one super-block of 256 values, one row, one lane group g)
// and register dequantisation into 8 bf16x8 B-fragments.
// ---------------------------------------------------------------------------

struct RawQ4K { u32x4 hdr, p0, p1; };
struct RawQ5K { u32x4 hdr, p0, p1, qh; };
struct RawQ6K { u32x4 qa, qb, qh; u32x4 sc; uint32_t d; };
struct RawQ8 { u32x4 q0, q1, q2, q3; uint32_t d; };
struct RawF16 { u32x4 v[8]; };
struct RawF32 { u32x4 v[16]; };

template <int T> struct RawOf;
template <> struct RawOf<QT_Q4_K> { typedef RawQ4K type; };
template <> struct RawOf<QT_Q5_K> { typedef RawQ5K type; };
template <> struct RawOf<QT_Q6_K> { typedef RawQ6K type; };
template <> struct RawOf<QT_Q8_0> { typedef RawQ8 type; };
template <> struct RawOf<QT_F16> { typedef RawF16 type; };
template <> struct RawOf<QT_BF16> { typedef RawF16 type; };
template <> struct RawOf<QT_F32> { typedef RawF32 type; };

// Geometry of a weight matrix on the device.
struct WDesc {
  const uint8_t* w;  // base pointer (format-specific layout, see top of file)
  int rows;          // R (padded to 16 in the tiled layout)
  int K;             // columns (multiple of 256)
};

template <int T> struct TileBytes;
template <> struct TileBytes<QT_Q4_K> { static constexpr int v = 2304; };
template <> struct TileBytes<QT_Q5_K> { static constexpr int v = 2816; };
template <> struct TileBytes<QT_Q6_K> { static constexpr int v = 3360; };
template <> struct TileBytes<QT_Q8_0> { static constexpr int v = 4352; };
template <> struct TileBytes<QT_F16> { static constexpr int v = 8192; };
template <> struct TileBytes<QT_BF16> { static constexpr int v = 8192; };
template <> struct TileBytes<QT_F32> { static constexpr int v = 16384; };

// base of the tile-block holding `row` (any row of the tile) at super-block sb
template <int T>
DEVI const uint8_t* tile_block(const WDesc& W, int row, int sb) {
  return W.w + ((size_t)(row >> 4) * (W.K >> 8) + sb) * TileBytes<T>::v;
}

// k offset (within the 256 super-block) of K-step t for lane group g
template <int T> DEVI int xoff(int t, int g);
template <> DEVI int xoff<QT_Q4_K>(int t, int g) {
  int c = (t < 4 ? 0 : 2) + (g >> 1);
  return 64 * c + 32 * ((t >> 1) & 1) + 16 * (g & 1) + 8 * (t & 1);
}
template <> DEVI int xoff<QT_Q5_K>(int t, int g) { return xoff<QT_Q4_K>(t, g); }
template <> DEVI int xoff<QT_Q6_K>(int t, int g) {
  return 128 * (g >> 1) + 32 * (t >> 1) + 16 * (g & 1) + 8 * (t & 1);
}
template <> DEVI int xoff<QT_Q8_0>(int t, int g) { return 64 * g + 8 * t; }
template <> DEVI int xoff<QT_F16>(int t, int g) { return 64 * g + 8 * t; }
template <> DEVI int xoff<QT_BF16>(int t, int g) { return 64 * g + 8 * t; }
template <> DEVI int xoff<QT_F32>(int t, int g) { return 64 * g + 8 * t; }

// ---- Q4_K -----------------------------------------------------------------
template <bool NT>
DEVI RawQ4K load_raw_q4k(const WDesc& W, int row, int sb, int g) {
  const uint8_t* b = tile_block<QT_Q4_K>(W, row, sb);
  const int r = row & 15, l = 16 * g + r;
  RawQ4K x;
  x.hdr = NT ? ld16_nt(b + 16 * r) : ld16(b + 16 * r);
  x.p0 = NT ? ld16_nt(b + 256 + 16 * l) : ld16(b + 256 + 16 * l);
  x.p1 = NT ? ld16_nt(b + 1280 + 16 * l) : ld16(b + 1280 + 16 * l);
  return x;
}

// 16 bytes of nibbles -> 4 K-steps (low 0-7, low 8-15, high 0-7, high 8-15)
DEVI void nib16_to_frags(u32x4 p, float a_lo, float m_lo, float a_hi, float m_hi, bf16x8* out) {
  float v[8];
#pragma unroll
  for (int half = 0; half < 2; ++half) {        // bytes 0-7 / 8-15
    uint32_t w0 = p[2 * half], w1 = p[2 * half + 1];
    uint32_t l0 = w0 & 0x0F0F0F0Fu, l1 = w1 & 0x0F0F0F0Fu;
    uint32_t h0 = (w0 >> 4) & 0x0F0F0F0Fu, h1 = (w1 >> 4) & 0x0F0F0F0Fu;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = a_lo * (float)((l0 >> (8 * i)) & 0xFF) - m_lo;
      v[4 + i] = a_lo * (float)((l1 >> (8 * i)) & 0xFF) - m_lo;
    }
    out[half] = pack8(v);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = a_hi * (float)((h0 >> (8 * i)) & 0xFF) - m_hi;
      v[4 + i] = a_hi * (float)((h1 >> (8 * i)) & 0xFF) - m_hi;
    }
    out[2 + half] = pack8(v);
  }
}

DEVI void deq_q4k(const RawQ4K& r, int g, bf16x8* wf) {
  const float d = h2f(r.hdr[0] & 0xFFFF), dmin = h2f(r.hdr[0] >> 16);
  const int c0 = g >> 1;
  int sc, m;
  float a[4], mm[4];
  const int js[4] = {2 * c0, 2 * c0 + 1, 4 + 2 * c0, 5 + 2 * c0};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i < 2) k4_scale_min_t<false>(js[i], r.hdr[1], r.hdr[2], r.hdr[3], sc, m);
    else k4_scale_min_t<true>(js[i], r.hdr[1], r.hdr[2], r.hdr[3], sc, m);
    a[i] = d * (float)sc;
    mm[i] = dmin * (float)m;
  }
  nib16_to_frags(r.p0, a[0], mm[0], a[1], mm[1], wf);
  nib16_to_frags(r.p1, a[2], mm[2], a[3], mm[3], wf + 4);
}

// ---- Q5_K -----------------------------------------------------------------
template <bool NT>
DEVI RawQ5K load_raw_q5k(const WDesc& W, int row, int sb, int g) {
  const uint8_t* b = tile_block<QT_Q5_K>(W, row, sb);
  const int r = row & 15, l = 16 * g + r;
  RawQ5K x;
  x.hdr = NT ? ld16_nt(b + 16 * r) : ld16(b + 16 * r);
  x.qh = NT ? ld16_nt(b + 256 + 16 * (16 * (g & 1) + r)) : ld16(b + 256 + 16 * (16 * (g & 1) + r));
  x.p0 = NT ? ld16_nt(b + 768 + 16 * l) : ld16(b + 768 + 16 * l);
  x.p1 = NT ? ld16_nt(b + 1792 + 16 * l) : ld16(b + 1792 + 16 * l);
  return x;
}

DEVI void nib16h_to_frags(u32x4 p, u32x4 qh, int c, float a_lo, float m_lo, float a_hi, float m_hi,
                          bf16x8* out) {
  float v[8];
  const int slo = 2 * c, shi = 2 * c + 1;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    uint32_t w[2] = {p[2 * half], p[2 * half + 1]};
    uint32_t h[2] = {qh[2 * half], qh[2 * half + 1]};
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t byte = (w[q] >> (8 * i)) & 0xFF;
        uint32_t hb = (h[q] >> (8 * i)) & 0xFF;
        v[4 * q + i] = a_lo * (float)((byte & 0xF) | (((hb >> slo) & 1) << 4)) - m_lo;
      }
    out[half] = pack8(v);
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t byte = (w[q] >> (8 * i)) & 0xFF;
        uint32_t hb = (h[q] >> (8 * i)) & 0xFF;
        v[4 * q + i] = a_hi * (float)((byte >> 4) | (((hb >> shi) & 1) << 4)) - m_hi;
      }
    out[2 + half] = pack8(v);
  }
}

DEVI void deq_q5k(const RawQ5K& r, int g, bf16x8* wf) {
  const float d = h2f(r.hdr[0] & 0xFFFF), dmin = h2f(r.hdr[0] >> 16);
  const int c0 = g >> 1, c1 = 2 + (g >> 1);
  int sc, m;
  float a[4], mm[4];
  const int js[4] = {2 * c0, 2 * c0 + 1, 2 * c1, 2 * c1 + 1};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i < 2) k4_scale_min_t<false>(js[i], r.hdr[1], r.hdr[2], r.hdr[3], sc, m);
    else k4_scale_min_t<true>(js[i], r.hdr[1], r.hdr[2], r.hdr[3], sc, m);
    a[i] = d * (float)sc;
    mm[i] = dmin * (float)m;
  }
  nib16h_to_frags(r.p0, r.qh, c0, a[0], mm[0], a[1], mm[1], wf);
  nib16h_to_frags(r.p1, r.qh, c1, a[2], mm[2], a[3], mm[3], wf + 4);
}

// ---- Q6_K ------------------------------------------------------------------
template <bool NT>
DEVI RawQ6K load_raw_q6k(const WDesc& W, int row, int sb, int g) {
  const uint8_t* b = tile_block<QT_Q6_K>(W, row, sb);
  const int r = row & 15, l = 16 * g + r;
  RawQ6K x;
  x.qa = NT ? ld16_nt(b + 16 * l) : ld16(b + 16 * l);
  x.qb = NT ? ld16_nt(b + 1024 + 16 * l) : ld16(b + 1024 + 16 * l);
  x.qh = NT ? ld16_nt(b + 2048 + 16 * l) : ld16(b + 2048 + 16 * l);
  x.sc = ld16(b + 3072 + 16 * r);
  x.d = *reinterpret_cast<const uint16_t*>(b + 3328 + 2 * r);
  return x;
}

DEVI void deq_q6k(const RawQ6K& r, int g, bf16x8* wf) {
  const float d = h2f((uint16_t)r.d);
  const int n = g >> 1, par = g & 1;
  float a[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    int idx = 8 * n + par + 2 * u;   // scale index
    int8_t s = (int8_t)((r.sc[idx >> 2] >> (8 * (idx & 3))) & 0xFF);
    a[u] = d * (float)s;
  }
  float v[8];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const u32x4 ql = (u & 1) ? r.qb : r.qa;
    const int nshift = (u >> 1) ? 4 : 0;     // q1,q2 low nibble; q3,q4 high nibble
    const int hshift = 2 * u;
#pragma unroll
    for (int s = 0; s < 2; ++s) {            // bytes 8s .. 8s+7 of the 16-byte range
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        uint32_t wl = ql[2 * s + q], wh = r.qh[2 * s + q];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int lo = (wl >> (8 * i + nshift)) & 0xF;
          int hi = (wh >> (8 * i + hshift)) & 3;
          v[4 * q + i] = a[u] * (float)((lo | (hi << 4)) - 32);
        }
      }
      wf[2 * u + s] = pack8(v);
    }
  }
}

// ---- per-K-step dequant (Q4_K / Q6_K): scales once per super-block, then one 8-value
// fragment per MFMA K-step, so a tile's 64 bf16 values never sit in registers at once
// (the large-M GEMM keeps RT weight tiles x MT activation tiles of accumulators live).
struct ScQ4K { float a[4], m[4]; };
struct ScQ6K { float a[4]; };

DEVI void prep_q4k(const RawQ4K& r, int g, ScQ4K& s) {
  const float d = h2f(r.hdr[0] & 0xFFFF), dmin = h2f(r.hdr[0] >> 16);
  const int c0 = g >> 1;
  const int js[4] = {2 * c0, 2 * c0 + 1, 4 + 2 * c0, 5 + 2 * c0};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int sc, m;
    if (i < 2) k4_scale_min_t<false>(js[i], r.hdr[1], r.hdr[2], r.hdr[3], sc, m);
    else k4_scale_min_t<true>(js[i], r.hdr[1], r.hdr[2], r.hdr[3], sc, m);
    s.a[i] = d * (float)sc;
    s.m[i] = dmin * (float)m;
  }
}

// fragment t of deq_q4k's output (t = 4*(p1) + 2*(high nibble) + half)
DEVI bf16x8 frag_q4k(const RawQ4K& r, const ScQ4K& s, int t) {
  const u32x4 p = t < 4 ? r.p0 : r.p1;
  const int half = t & 1, hi = (t >> 1) & 1, si = (t < 4 ? 0 : 2) + hi;
  const uint32_t w0 = p[2 * half], w1 = p[2 * half + 1];
  const int sh = 4 * hi;
  float v[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = s.a[si] * (float)((w0 >> (8 * i + sh)) & 0xF) - s.m[si];
    v[4 + i] = s.a[si] * (float)((w1 >> (8 * i + sh)) & 0xF) - s.m[si];
  }
  return pack8(v);
}

DEVI void prep_q6k(const RawQ6K& r, int g, ScQ6K& s) {
  const float d = h2f((uint16_t)r.d);
  const int n = g >> 1, par = g & 1;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int idx = 8 * n + par + 2 * u;
    const int8_t sc = (int8_t)((r.sc[idx >> 2] >> (8 * (idx & 3))) & 0xFF);
    s.a[u] = d * (float)sc;
  }
}

// fragment t of deq_q6k's output (t = 2*u + s)
DEVI bf16x8 frag_q6k(const RawQ6K& r, const ScQ6K& sc, int t) {
  const int u = t >> 1, sidx = t & 1;
  const u32x4 ql = (u & 1) ? r.qb : r.qa;
  const int nshift = (u >> 1) ? 4 : 0, hshift = 2 * u;
  float v[8];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const uint32_t wl = ql[2 * sidx + q], wh = r.qh[2 * sidx + q];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int lo = (wl >> (8 * i + nshift)) & 0xF;
      const int hi = (wh >> (8 * i + hshift)) & 3;
      v[4 * q + i] = sc.a[u] * (float)((lo | (hi << 4)) - 32);
    }
  }
  return pack8(v);
}

template <int T> struct ScOf { typedef int type; };
template <> struct ScOf<QT_Q4_K> { typedef ScQ4K type; };
template <> struct ScOf<QT_Q6_K> { typedef ScQ6K type; };
template <int T> constexpr bool kPerStep = (T == QT_Q4_K || T == QT_Q6_K);

template <int T>
DEVI void prep_sc(const typename RawOf<T>::type& r, int g, typename ScOf<T>::type& s) {
  if constexpr (T == QT_Q4_K) prep_q4k(r, g, s);
  else if constexpr (T == QT_Q6_K) prep_q6k(r, g, s);
}
template <int T>
DEVI bf16x8 frag_t(const typename RawOf<T>::type& r, const typename ScOf<T>::type& s, int t) {
  if constexpr (T == QT_Q4_K) return frag_q4k(r, s, t);
  else return frag_q6k(r, s, t);
}

// ---- Q8_0 ------------------------------------------------------------------
template <bool NT>
DEVI RawQ8 load_raw_q8(const WDesc& W, int row, int sb, int g) {
  const uint8_t* b = tile_block<QT_Q8_0>(W, row, sb);
  const int r = row & 15, l = 16 * g + r;
  RawQ8 x;
  x.q0 = NT ? ld16_nt(b + 16 * l) : ld16(b + 16 * l);
  x.q1 = NT ? ld16_nt(b + 1024 + 16 * l) : ld16(b + 1024 + 16 * l);
  x.q2 = NT ? ld16_nt(b + 2048 + 16 * l) : ld16(b + 2048 + 16 * l);
  x.q3 = NT ? ld16_nt(b + 3072 + 16 * l) : ld16(b + 3072 + 16 * l);
  x.d = *reinterpret_cast<const uint32_t*>(b + 4096 + 16 * r + 4 * g);
  return x;
}

DEVI void deq_q8(const RawQ8& r, int g, bf16x8* wf) {
  const float d0 = h2f(r.d & 0xFFFF), d1 = h2f(r.d >> 16);
  const u32x4 q[4] = {r.q0, r.q1, r.q2, r.q3};
  float v[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const float d = t < 4 ? d0 : d1;
    uint32_t w0 = q[t >> 1][2 * (t & 1)], w1 = q[t >> 1][2 * (t & 1) + 1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = d * (float)(int8_t)((w0 >> (8 * i)) & 0xFF);
      v[4 + i] = d * (float)(int8_t)((w1 >> (8 * i)) & 0xFF);
    }
    wf[t] = pack8(v);
  }
}

// ---- plain F16 / BF16 / F32 ---------------------------------------------------
template <bool NT>
DEVI RawF16 load_raw_f16(const WDesc& W, int row, int sb, int g) {
  const uint8_t* b = tile_block<QT_F16>(W, row, sb);
  const int l = 16 * g + (row & 15);
  RawF16 x;
#pragma unroll
  for (int t = 0; t < 8; ++t) x.v[t] = NT ? ld16_nt(b + 1024 * t + 16 * l) : ld16(b + 1024 * t + 16 * l);
  return x;
}
DEVI void deq_bf16(const RawF16& r, int g, bf16x8* wf) {
#pragma unroll
  for (int t = 0; t < 8; ++t) wf[t] = __builtin_bit_cast(bf16x8, r.v[t]);
}
DEVI void deq_f16(const RawF16& r, int g, bf16x8* wf) {
  float v[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = h2f(r.v[t][i] & 0xFFFF);
      v[2 * i + 1] = h2f(r.v[t][i] >> 16);
    }
    wf[t] = pack8(v);
  }
}
template <bool NT>
DEVI RawF32 load_raw_f32(const WDesc& W, int row, int sb, int g) {
  const uint8_t* b = tile_block<QT_F32>(W, row, sb);
  const int l = 16 * g + (row & 15);
  RawF32 x;
#pragma unroll
  for (int t = 0; t < 16; ++t) x.v[t] = NT ? ld16_nt(b + 1024 * t + 16 * l) : ld16(b + 1024 * t + 16 * l);
  return x;
}
DEVI void deq_f32(const RawF32& r, int g, bf16x8* wf) {
  float v[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // NB: copy the vector element out first; __builtin_bit_cast on an ext_vector
      // element lvalue returns element 0 with hipcc (ROCm 7.2).
      const uint32_t u0 = r.v[2 * t][i], u1 = r.v[2 * t + 1][i];
      v[i] = __uint_as_float(u0);
      v[4 + i] = __uint_as_float(u1);
    }
    wf[t] = pack8(v);
  }
}

// ---- uniform dispatch ---------------------------------------------------------
template <int T, bool NT>
DEVI typename RawOf<T>::type load_raw(const WDesc& W, int row, int sb, int g) {
  if constexpr (T == QT_Q4_K) return load_raw_q4k<NT>(W, row, sb, g);
  else if constexpr (T == QT_Q5_K) return load_raw_q5k<NT>(W, row, sb, g);
  else if constexpr (T == QT_Q6_K) return load_raw_q6k<NT>(W, row, sb, g);
  else if constexpr (T == QT_Q8_0) return load_raw_q8<NT>(W, row, sb, g);
  else if constexpr (T == QT_F16 || T == QT_BF16) return load_raw_f16<NT>(W, row, sb, g);
  else return load_raw_f32<NT>(W, row, sb, g);
}

template <int T>
DEVI void dequant(const typename RawOf<T>::type& r, int g, bf16x8* wf) {
  if constexpr (T == QT_Q4_K) deq_q4k(r, g, wf);
  else if constexpr (T == QT_Q5_K) deq_q5k(r, g, wf);
  else if constexpr (T == QT_Q6_K) deq_q6k(r, g, wf);
  else if constexpr (T == QT_Q8_0) deq_q8(r, g, wf);
  else if constexpr (T == QT_F16) deq_f16(r, g, wf);
  else if constexpr (T == QT_BF16) deq_bf16(r, g, wf);
  else deq_f32(r, g, wf);
}

// Scalar dequant of element k of a row (embedding gather; not a hot path).
DEVI float dequant_elem(const WDesc& W, int type, int row, int k) {
  const int nb = W.K >> 8;
  switch (type) {
    case QT_F32: return reinterpret_cast<const float*>(W.w)[(size_t)row * W.K + k];
    case QT_F16: return h2f(reinterpret_cast<const uint16_t*>(W.w)[(size_t)row * W.K + k]);
    case QT_BF16: return bf2f(reinterpret_cast<const uint16_t*>(W.w)[(size_t)row * W.K + k]);
    case QT_Q8_0: {
      int8_t q = (int8_t)W.w[(size_t)row * W.K + k];
      const uint16_t* dp = reinterpret_cast<const uint16_t*>(W.w + (size_t)W.rows * W.K);
      return h2f(dp[(size_t)row * (W.K >> 5) + (k >> 5)]) * (float)q;
    }
    case QT_Q4_K:
    case QT_Q5_K: {
      const int bs = type == QT_Q4_K ? 144 : 176;
      const uint8_t* b = W.w + ((size_t)row * nb + (k >> 8)) * bs;
      const int kk = k & 255, c = kk >> 6, hi = (kk >> 5) & 1, l = kk & 31;
      const uint32_t* h = reinterpret_cast<const uint32_t*>(b);
      int sc, m;
      k4_scale_min(2 * c + hi, h[1], h[2], h[3], sc, m);
      const uint8_t* qs = b + (type == QT_Q4_K ? 16 : 48);
      int q = hi ? (qs[32 * c + l] >> 4) : (qs[32 * c + l] & 0xF);
      if (type == QT_Q5_K) q |= ((b[16 + l] >> (2 * c + hi)) & 1) << 4;
      return h2f(h[0] & 0xFFFF) * sc * q - h2f(h[0] >> 16) * m;
    }
    case QT_Q6_K: {
      const size_t nblk = (size_t)W.rows * nb, bi = (size_t)row * nb + (k >> 8);
      const uint8_t* ql = W.w + bi * 128;
      const uint8_t* qh = W.w + nblk * 128 + bi * 64;
      const int8_t* sc = reinterpret_cast<const int8_t*>(W.w + nblk * 192 + bi * 16);
      const float d = h2f(reinterpret_cast<const uint16_t*>(W.w + nblk * 208)[bi]);
      const int kk = k & 255, n = kk >> 7, r = kk & 127, u = r >> 5, l = r & 31;
      const uint8_t qlb = ql[64 * n + l + 32 * (u & 1)];
      const int lo = (u >> 1) ? (qlb >> 4) : (qlb & 0xF);
      const int hi = (qh[32 * n + l] >> (2 * u)) & 3;
      return d * (float)sc[8 * n + (l >> 4) + 2 * u] * (float)((lo | (hi << 4)) - 32);
    }
  }
  return 0.f;
}
