// Shared device helpers for the gfx950 (CDNA4) kernels of nats_llm_studio_amd.
//
// Weight formats live on the device in GGUF block encodings (never pre-dequantised:
// decode is HBM-bound), re-tiled at load time ("tiled" layout, same bytes):
//   rows are padded to 16 and grouped into 16-row tiles; for every (tile, 256-value
//   super-block) the 16 rows' blocks form ONE contiguous "tile-block" of TB bytes,
//   arranged so that each wave-wide 16-B load instruction reads 1 KiB contiguous
//   (lane l = 16*g + r -> byte 16*l of a 1 KiB piece). Tile-blocks are ordered
//   [tile][super-block], so a wave walking K streams sequential memory.
//
// Every format uses the SAME lane -> k map: K-step t (0..7) of lane group g covers
// k = 32*t + 8*g .. +8 of the super-block (so a K-step is one 32-wide MFMA K slice and
// each 64-wide quarter of a super-block is spread evenly over all 64 lanes: the LDS-W
// GEMM dequantises quarter q with every lane busy). Per (g, r) the pieces hold:
//     Q4_K  TB=2304: hdr[r] (16) | P_h[g][r] (16) h=0,1: qs bytes 8g..8g+7 of chunks 2h, 2h+1
//     Q5_K  TB=2816: hdr[r] | QH[g][r] (8): qh bytes 8g..8g+7 | P_0 | P_1
//     Q6_K  TB=3360: QL_n[g][r] (16) n=0,1: ql[64n+8g..+8] | ql[64n+32+8g..+8]
//                    | QH[g][r] (16): qh[8g..+8] | qh[32+8g..+8] | sc[r] (16) | d[r] (2)
//     Q8_0  TB=4352: Q_p[g][r] (16) p=0..3: blocks 2p, 2p+1, bytes 8g..8g+7 | d[r][8] (f16)
//     F16/BF16 TB=8192: v[t][g][r] (16);  F32 TB=16384: v[t][half][g][r] (16)
// Embedding tables keep a row-major "rows" layout (gathered, not streamed):
//   Q4_K/Q5_K native blocks; Q6_K planes ql|qh|sc|d; Q8_0 planes qs|d.
//
// Activations (every GEMM/GEMV input) are f16 (`act_t`) and the matrix cores run
// v_mfma_f32_16x16x32_f16: lane l = 16*g + r holds A[row r][k = 8g + j] and
// B[k = 8g + j][col r], j = 0..7. K-quant values are integers < 256, so they are
// dequantised with the f16 "magic number" trick: v_perm_b32 places byte b under the
// exponent byte 0x64 -> f16 (1024 + b) exactly, then one packed subtract (exact) and one
// packed FMA with the sub-block scale (single rounding) give d*sc*q - dmin*m, two values
// per instruction. Q4_K's 4-bit values skip the subtract: read as fp8 e4m3 a byte < 16 is
// exactly b * 2^-9, so one scaled fp8 -> f16 conversion per pair yields b (frag8_nib).
// The residual stream and all accumulators stay fp32.
#pragma once
#include <type_traits>
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 act_t;   // activation dtype of GEMM operands (torch.float16 on the host)

enum QType : int {
  QT_F32 = 0, QT_F16 = 1, QT_Q8_0 = 8, QT_Q4_K = 12, QT_Q5_K = 13, QT_Q6_K = 14, QT_BF16 = 30,
  // device-only: the 32-value affine blocks of ggml Q4_0 / Q4_1 / Q5_0 / Q5_1 (x = d*q + m, q 5-bit; the
  // symmetric types with m = -8d / -16d, exact) in the Q5_K tile layout with per-block f16 (d, m)
  QT_Q51 = 101
};

#define DEVI __device__ __forceinline__

// Q4_K nibbles -> f16 through the scaled fp8 conversion (frag8_nib) instead of the magic-number subtract;
// -DNLS_Q4_FP8CVT=0 builds the previous form (A/B builds, tools/gemm_ab.py; profiles/q4_fp8cvt_ab_r05.txt)
#ifndef NLS_Q4_FP8CVT
#define NLS_Q4_FP8CVT 1
#endif

DEVI float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
DEVI float bf2f(uint16_t b) { return __builtin_bit_cast(float, ((uint32_t)b) << 16); }
DEVI uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

DEVI u32x4 ld16(const void* p) { return *reinterpret_cast<const u32x4*>(p); }

// Paged KV cache element types: bf16 (default) or OCP fp8 e4m3 (NLS_KV_DTYPE=fp8: half the bytes per
// decode step). raw = what one lane loads for 8 dims (kept in flight by the attention prefetch);
// bf16() unpacks it to 8 bf16 (u32x4) -- exact for fp8 (3 mantissa bits fit bf16's 7).
template <typename KV> struct KVRaw;
template <> struct KVRaw<__bf16> {
  typedef u32x4 raw;
  static DEVI raw ld(const __bf16* p) { return ld16(p); }
  static DEVI u32x4 bf16(const raw& r) { return r; }
};
template <> struct KVRaw<uint8_t> {
  typedef uint2 raw;
  static DEVI raw ld(const uint8_t* p) { return *reinterpret_cast<const uint2*>(p); }
  static DEVI u32x4 bf16(const raw& r) {
    // bytes 2i, 2i+1 -> dword i (bf16 pair): one packed scaled conversion (scale 1) per pair, exact (e4m3's
    // 3 mantissa bits and its exponent range fit bf16)
    auto cv = [](uint32_t w, auto hi) {
      return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w, 1.f, decltype(hi)::value));
    };
    typedef std::integral_constant<bool, false> lo_w;
    typedef std::integral_constant<bool, true> hi_w;
    return u32x4{cv(r.x, lo_w{}), cv(r.x, hi_w{}), cv(r.y, lo_w{}), cv(r.y, hi_w{})};
  }
};
// 4 values -> the cache (fp8: saturated to +-448, the e4m3 range)
DEVI void kv_st4(__bf16* d, float a, float b, float c, float e) {
  typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
  *reinterpret_cast<bf4*>(d) = bf4{(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)e};
}
DEVI void kv_st4(uint8_t* d, float a, float b, float c, float e) {
  auto sat = [](float v) { return fminf(fmaxf(v, -448.f), 448.f); };
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(a), sat(b), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(c), sat(e), w, true);
  *reinterpret_cast<int*>(d) = w;
}
DEVI u32x4 ld16_nt(const void* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}
DEVI u32x2 ld8(const void* p) { return *reinterpret_cast<const u32x2*>(p); }
DEVI u32x2 ld8_nt(const void* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
}

DEVI f32x4 mfma16(const f16x8& a, const f16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// ---- f16 magic-number helpers -------------------------------------------------------
DEVI f16x2 as_h2(uint32_t u) { return __builtin_bit_cast(f16x2, u); }
DEVI uint32_t as_u32(f16x2 h) { return __builtin_bit_cast(uint32_t, h); }
DEVI f16x2 h2(_Float16 v) { return f16x2{v, v}; }
// bytes 0,1 (mag_lo) / 2,3 (mag_hi) of w -> f16 pair (1024 + b_i), exact for b_i < 1024
DEVI f16x2 mag_lo(uint32_t w) { return as_h2(__builtin_amdgcn_perm(0x64646464u, w, 0x04010400u)); }
DEVI f16x2 mag_hi(uint32_t w) { return as_h2(__builtin_amdgcn_perm(0x64646464u, w, 0x04030402u)); }

// 8 small unsigned ints (bytes of n0, n1) -> f16x8 of a*(b - off0) + c.  `off` = 1024 + the
// format's zero point (exact), then one FMA: a single rounding per value.
DEVI f16x8 frag8(uint32_t n0, uint32_t n1, f16x2 off, f16x2 a, f16x2 c) {
  u32x4 u;
  u[0] = as_u32(__builtin_elementwise_fma(mag_lo(n0) - off, a, c));
  u[1] = as_u32(__builtin_elementwise_fma(mag_hi(n0) - off, a, c));
  u[2] = as_u32(__builtin_elementwise_fma(mag_lo(n1) - off, a, c));
  u[3] = as_u32(__builtin_elementwise_fma(mag_hi(n1) - off, a, c));
  return __builtin_bit_cast(f16x8, u);
}
// 8 nibble values (bytes of n0, n1, each < 16) -> f16x8 of a*b + c, two values per conversion: a byte b < 16
// read as OCP fp8 e4m3 is exactly b * 2^-9 (0..7 subnormal, 8..15 exponent field 1), so gfx950's scaled
// fp8 -> f16 conversion with scale 2^9 yields b itself and the FMA follows directly -- the magic-number
// path's exact (1024 + b) - 1024 subtract is gone (4 of its 12 VALU ops per 8 values). Same single rounding,
// bit-identical to frag8 with off = 1024.
DEVI f16x2 nib_h2(uint32_t w, bool hi) {
  return hi ? __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w, 512.f, true)
            : __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w, 512.f, false);
}
DEVI f16x8 frag8_nib(uint32_t n0, uint32_t n1, f16x2 a, f16x2 c) {
  u32x4 u;
  u[0] = as_u32(__builtin_elementwise_fma(nib_h2(n0, false), a, c));
  u[1] = as_u32(__builtin_elementwise_fma(nib_h2(n0, true), a, c));
  u[2] = as_u32(__builtin_elementwise_fma(nib_h2(n1, false), a, c));
  u[3] = as_u32(__builtin_elementwise_fma(nib_h2(n1, true), a, c));
  return __builtin_bit_cast(f16x8, u);
}
// 4 bytes -> two f16 pairs (b - off) (exact small integers), e.g. 6-bit scales
DEVI void bytes_to_h(uint32_t w, f16x2 off, f16x2& lo, f16x2& hi) {
  lo = mag_lo(w) - off;
  hi = mag_hi(w) - off;
}

// ---------------------------------------------------------------------------
// Per-format raw loads (one super-block of 256 values, one row, one lane group g),
// per-super-block scale preparation, and per-K-step fragments.
// ---------------------------------------------------------------------------

struct RawQ4K { u32x4 hdr, p0, p1; };
struct RawQ5K { u32x4 hdr, p0, p1; u32x2 qh; };
struct RawQ51 { u32x4 dd, mm, p0, p1; u32x2 qh; };
struct RawQ6K { u32x4 qa, qb, qh; u32x4 sc; uint32_t d; };
struct RawQ8 { u32x4 q[4]; u32x4 d; };
struct RawF16 { u32x4 v[8]; };
struct RawF32 { u32x4 v[16]; };

template <int T> struct RawOf;
template <> struct RawOf<QT_Q4_K> { typedef RawQ4K type; };
template <> struct RawOf<QT_Q5_K> { typedef RawQ5K type; };
template <> struct RawOf<QT_Q51> { typedef RawQ51 type; };
template <> struct RawOf<QT_Q6_K> { typedef RawQ6K type; };
template <> struct RawOf<QT_Q8_0> { typedef RawQ8 type; };
template <> struct RawOf<QT_F16> { typedef RawF16 type; };
template <> struct RawOf<QT_BF16> { typedef RawF16 type; };
template <> struct RawOf<QT_F32> { typedef RawF32 type; };

// Per-super-block scales of one row, as f16 pairs (a2[i] = scales 2i, 2i+1; kept as packed
// vectors: arrays of scalar halves end up in scratch): value = a[s] * q + c[s] for sub-scale s.
struct ScK { f16x2 a2[4], c2[4]; };          // Q4_K / Q5_K: s = K-step t (32-value sub-blocks)
struct ScQ6K { f16x2 a2[4]; };               // Q6_K: 16-value sub-blocks, lane-dependent index
struct ScQ8 { f16x2 a2[4]; };                // Q8_0: block t
struct ScNone { };
// broadcast scale s (compile-time after unrolling) of a packed array
DEVI f16x2 bcast(const f16x2* a2, int s) {
  const f16x2 p = a2[s >> 1];
  return (s & 1) ? __builtin_shufflevector(p, p, 1, 1) : __builtin_shufflevector(p, p, 0, 0);
}

template <int T> struct ScOf { typedef ScNone type; };
template <> struct ScOf<QT_Q4_K> { typedef ScK type; };
template <> struct ScOf<QT_Q5_K> { typedef ScK type; };
template <> struct ScOf<QT_Q51> { typedef ScK type; };
template <> struct ScOf<QT_Q6_K> { typedef ScQ6K type; };
template <> struct ScOf<QT_Q8_0> { typedef ScQ8 type; };

// Geometry of a weight matrix on the device.
struct WDesc {
  const uint8_t* w;  // base pointer (format-specific layout, see top of file)
  int rows;          // R (padded to 16 in the tiled layout)
  int K;             // columns (multiple of 256)
};

template <int T> struct TileBytes;
template <> struct TileBytes<QT_Q4_K> { static constexpr int v = 2304; };
template <> struct TileBytes<QT_Q5_K> { static constexpr int v = 2816; };
template <> struct TileBytes<QT_Q51> { static constexpr int v = 3072; };
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

// k offset (within the 256 super-block) of K-step t for lane group g: the same for all formats
template <int T> DEVI int xoff(int t, int g) { return 32 * t + 8 * g; }

// ---- Q4_K / Q5_K ---------------------------------------------------------------
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
template <bool NT>
DEVI RawQ5K load_raw_q5k(const WDesc& W, int row, int sb, int g) {
  const uint8_t* b = tile_block<QT_Q5_K>(W, row, sb);
  const int r = row & 15, l = 16 * g + r;
  RawQ5K x;
  x.hdr = NT ? ld16_nt(b + 16 * r) : ld16(b + 16 * r);
  x.qh = NT ? ld8_nt(b + 256 + 8 * l) : ld8(b + 256 + 8 * l);
  x.p0 = NT ? ld16_nt(b + 768 + 16 * l) : ld16(b + 768 + 16 * l);
  x.p1 = NT ? ld16_nt(b + 1792 + 16 * l) : ld16(b + 1792 + 16 * l);
  return x;
}

// Q51 tile-block: [16 rows x (8 f16 d | 8 f16 m)] 512 B | QH as Q5_K 512 B | P as Q5_K 2048 B
template <bool NT>
DEVI RawQ51 load_raw_q51(const WDesc& W, int row, int sb, int g) {
  const uint8_t* b = tile_block<QT_Q51>(W, row, sb);
  const int r = row & 15, l = 16 * g + r;
  RawQ51 x;
  x.dd = ld16(b + 32 * r);
  x.mm = ld16(b + 32 * r + 16);
  x.qh = NT ? ld8_nt(b + 512 + 8 * l) : ld8(b + 512 + 8 * l);
  x.p0 = NT ? ld16_nt(b + 1024 + 16 * l) : ld16(b + 1024 + 16 * l);
  x.p1 = NT ? ld16_nt(b + 2048 + 16 * l) : ld16(b + 2048 + 16 * l);
  return x;
}
// block t's (d, m) are the scale pair of K-step t: no unpacking
DEVI void prep_q51(const RawQ51& r, ScK& s) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    s.a2[i] = as_h2(r.dd[i]);
    s.c2[i] = as_h2(r.mm[i]);
  }
}
// the Q5_K nibble / high-bit arrangement (the loader re-packs the 32-blocks that way)
DEVI f16x8 frag_q51(const RawQ51& r, const ScK& s, int t) {
  const u32x4 p = t < 4 ? r.p0 : r.p1;
  const int wi = 2 * ((t >> 1) & 1), sh = 4 * (t & 1);
  const uint32_t n0 = ((p[wi] >> sh) & 0x0F0F0F0Fu) | (((r.qh[0] >> t) & 0x01010101u) << 4);
  const uint32_t n1 = ((p[wi + 1] >> sh) & 0x0F0F0F0Fu) | (((r.qh[1] >> t) & 0x01010101u) << 4);
  return frag8(n0, n1, h2((_Float16)1024.f), bcast(s.a2, t), bcast(s.c2, t));
}

// ggml get_scale_min_k4 for all 8 sub-blocks at once (bytes of 3 dwords), then f16:
// a[s] = d * sc[s], c[s] = -dmin * m[s]
DEVI void prep_kquant(const u32x4& hdr, ScK& s) {
  const uint32_t s0 = hdr[1], s1 = hdr[2], s2 = hdr[3];
  const uint32_t sc_lo = s0 & 0x3F3F3F3Fu, m_lo = s1 & 0x3F3F3F3Fu;
  const uint32_t sc_hi = (s2 & 0x0F0F0F0Fu) | ((s0 >> 2) & 0x30303030u);
  const uint32_t m_hi = ((s2 >> 4) & 0x0F0F0F0Fu) | ((s1 >> 2) & 0x30303030u);
  const f16x2 d = h2(__builtin_bit_cast(_Float16, (uint16_t)(hdr[0] & 0xFFFF)));
  const f16x2 nd = -h2(__builtin_bit_cast(_Float16, (uint16_t)(hdr[0] >> 16)));
  const f16x2 k1024 = h2((_Float16)1024.f);
  f16x2 v[4];
  bytes_to_h(sc_lo, k1024, v[0], v[1]);
  bytes_to_h(sc_hi, k1024, v[2], v[3]);
#pragma unroll
  for (int i = 0; i < 4; ++i) s.a2[i] = v[i] * d;
  bytes_to_h(m_lo, k1024, v[0], v[1]);
  bytes_to_h(m_hi, k1024, v[2], v[3]);
#pragma unroll
  for (int i = 0; i < 4; ++i) s.c2[i] = v[i] * nd;
}

// K-step t of Q4_K: chunk c = t >> 1 (in piece h = t >> 2, words 2*((t>>1)&1) +{0,1}), nibble t & 1
DEVI f16x8 frag_q4k(const RawQ4K& r, const ScK& s, int t) {
  const u32x4 p = t < 4 ? r.p0 : r.p1;
  const int wi = 2 * ((t >> 1) & 1), sh = 4 * (t & 1);
  const uint32_t n0 = (p[wi] >> sh) & 0x0F0F0F0Fu, n1 = (p[wi + 1] >> sh) & 0x0F0F0F0Fu;
#if NLS_Q4_FP8CVT
  return frag8_nib(n0, n1, bcast(s.a2, t), bcast(s.c2, t));
#else
  return frag8(n0, n1, h2((_Float16)1024.f), bcast(s.a2, t), bcast(s.c2, t));
#endif
}
// Q5_K: plus the 5th bit = bit t of the lane's 8 qh bytes
DEVI f16x8 frag_q5k(const RawQ5K& r, const ScK& s, int t) {
  const u32x4 p = t < 4 ? r.p0 : r.p1;
  const int wi = 2 * ((t >> 1) & 1), sh = 4 * (t & 1);
  const uint32_t n0 = ((p[wi] >> sh) & 0x0F0F0F0Fu) | (((r.qh[0] >> t) & 0x01010101u) << 4);
  const uint32_t n1 = ((p[wi + 1] >> sh) & 0x0F0F0F0Fu) | (((r.qh[1] >> t) & 0x01010101u) << 4);
  return frag8(n0, n1, h2((_Float16)1024.f), bcast(s.a2, t), bcast(s.c2, t));
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
// scale of K-step t for lane group g: int8 sc[2t + (g >> 1)] * d
DEVI void prep_q6k(const RawQ6K& r, int g, ScQ6K& s) {
  const uint32_t sel = (g >> 1) ? 0x07050301u : 0x06040200u;   // odd / even bytes of two dwords
  const uint32_t e0 = __builtin_amdgcn_perm(r.sc[1], r.sc[0], sel) ^ 0x80808080u;   // t = 0..3
  const uint32_t e1 = __builtin_amdgcn_perm(r.sc[3], r.sc[2], sel) ^ 0x80808080u;   // t = 4..7
  const f16x2 d = h2(__builtin_bit_cast(_Float16, (uint16_t)(r.d & 0xFFFF)));
  const f16x2 off = h2((_Float16)1152.f);     // 1024 + 128 (int8 via xor 0x80)
  f16x2 v[4];
  bytes_to_h(e0, off, v[0], v[1]);
  bytes_to_h(e1, off, v[2], v[3]);
#pragma unroll
  for (int i = 0; i < 4; ++i) s.a2[i] = v[i] * d;
}
// K-step t: n = t >> 2 (ql piece), low/high nibble (t >> 1) & 1, ql run t & 1, qh bits 2*(t & 3)
DEVI f16x8 frag_q6k(const RawQ6K& r, const ScQ6K& s, int t) {
  const u32x4 ql = t < 4 ? r.qa : r.qb;
  const int wi = 2 * (t & 1), sh = 4 * ((t >> 1) & 1), hs = 2 * (t & 3), hw = 2 * (t >> 2);
  const uint32_t n0 = ((ql[wi] >> sh) & 0x0F0F0F0Fu) | (((r.qh[hw] >> hs) & 0x03030303u) << 4);
  const uint32_t n1 = ((ql[wi + 1] >> sh) & 0x0F0F0F0Fu) | (((r.qh[hw + 1] >> hs) & 0x03030303u) << 4);
  return frag8(n0, n1, h2((_Float16)1056.f), bcast(s.a2, t), h2((_Float16)0.f));
}

// ---- Q8_0 ------------------------------------------------------------------
template <bool NT>
DEVI RawQ8 load_raw_q8(const WDesc& W, int row, int sb, int g) {
  const uint8_t* b = tile_block<QT_Q8_0>(W, row, sb);
  const int r = row & 15, l = 16 * g + r;
  RawQ8 x;
#pragma unroll
  for (int p = 0; p < 4; ++p) x.q[p] = NT ? ld16_nt(b + 1024 * p + 16 * l) : ld16(b + 1024 * p + 16 * l);
  x.d = ld16(b + 4096 + 16 * r);
  return x;
}
DEVI void prep_q8(const RawQ8& r, ScQ8& s) {
#pragma unroll
  for (int i = 0; i < 4; ++i) s.a2[i] = as_h2(r.d[i]);
}
DEVI f16x8 frag_q8(const RawQ8& r, const ScQ8& s, int t) {
  const u32x4 p = r.q[t >> 1];
  const int wi = 2 * (t & 1);
  return frag8(p[wi] ^ 0x80808080u, p[wi + 1] ^ 0x80808080u, h2((_Float16)1152.f), bcast(s.a2, t),
               h2((_Float16)0.f));
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
template <bool NT>
DEVI RawF32 load_raw_f32(const WDesc& W, int row, int sb, int g) {
  const uint8_t* b = tile_block<QT_F32>(W, row, sb);
  const int l = 16 * g + (row & 15);
  RawF32 x;
#pragma unroll
  for (int t = 0; t < 16; ++t) x.v[t] = NT ? ld16_nt(b + 1024 * t + 16 * l) : ld16(b + 1024 * t + 16 * l);
  return x;
}
DEVI f16x8 frag_f16(const RawF16& r, int t) { return __builtin_bit_cast(f16x8, r.v[t]); }
DEVI f16x8 frag_bf16(const RawF16& r, int t) {
  f16x8 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t u = r.v[t][i];
    o[2 * i] = (_Float16)__uint_as_float(u << 16);
    o[2 * i + 1] = (_Float16)__uint_as_float(u & 0xFFFF0000u);
  }
  return o;
}
DEVI f16x8 frag_f32(const RawF32& r, int t) {
  f16x8 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    // NB: copy the vector element out first; __builtin_bit_cast on an ext_vector
    // element lvalue returns element 0 with hipcc (ROCm 7.2).
    const uint32_t u0 = r.v[2 * t][i], u1 = r.v[2 * t + 1][i];
    o[i] = (_Float16)__uint_as_float(u0);
    o[4 + i] = (_Float16)__uint_as_float(u1);
  }
  return o;
}

// ---- uniform dispatch ---------------------------------------------------------
template <int T, bool NT>
DEVI typename RawOf<T>::type load_raw(const WDesc& W, int row, int sb, int g) {
  if constexpr (T == QT_Q4_K) return load_raw_q4k<NT>(W, row, sb, g);
  else if constexpr (T == QT_Q5_K) return load_raw_q5k<NT>(W, row, sb, g);
  else if constexpr (T == QT_Q51) return load_raw_q51<NT>(W, row, sb, g);
  else if constexpr (T == QT_Q6_K) return load_raw_q6k<NT>(W, row, sb, g);
  else if constexpr (T == QT_Q8_0) return load_raw_q8<NT>(W, row, sb, g);
  else if constexpr (T == QT_F16 || T == QT_BF16) return load_raw_f16<NT>(W, row, sb, g);
  else return load_raw_f32<NT>(W, row, sb, g);
}

// scales of one super-block (once), then frag_t(t) per K-step
template <int T>
DEVI void prep_sc(const typename RawOf<T>::type& r, int g, typename ScOf<T>::type& s) {
  if constexpr (T == QT_Q4_K || T == QT_Q5_K) prep_kquant(r.hdr, s);
  else if constexpr (T == QT_Q51) prep_q51(r, s);
  else if constexpr (T == QT_Q6_K) prep_q6k(r, g, s);
  else if constexpr (T == QT_Q8_0) prep_q8(r, s);
}
template <int T>
DEVI f16x8 frag_t(const typename RawOf<T>::type& r, const typename ScOf<T>::type& s, int t) {
  if constexpr (T == QT_Q4_K) return frag_q4k(r, s, t);
  else if constexpr (T == QT_Q5_K) return frag_q5k(r, s, t);
  else if constexpr (T == QT_Q51) return frag_q51(r, s, t);
  else if constexpr (T == QT_Q6_K) return frag_q6k(r, s, t);
  else if constexpr (T == QT_Q8_0) return frag_q8(r, s, t);
  else if constexpr (T == QT_F16) return frag_f16(r, t);
  else if constexpr (T == QT_BF16) return frag_bf16(r, t);
  else return frag_f32(r, t);
}
// all 8 K-step fragments of a super-block
template <int T>
DEVI void dequant(const typename RawOf<T>::type& r, int g, f16x8* wf) {
  typename ScOf<T>::type s;
  prep_sc<T>(r, g, s);
#pragma unroll
  for (int t = 0; t < 8; ++t) wf[t] = frag_t<T>(r, s, t);
}

// ggml get_scale_min_k4 (scalar; embedding gather only)
DEVI int byte_of(uint32_t s0, uint32_t s1, uint32_t s2, int i) {
  uint32_t w = i < 4 ? s0 : (i < 8 ? s1 : s2);
  return (w >> (8 * (i & 3))) & 0xFF;
}
DEVI void k4_scale_min(int j, uint32_t s0, uint32_t s1, uint32_t s2, int& sc, int& m) {
  if (j < 4) {
    sc = byte_of(s0, s1, s2, j) & 63;
    m = byte_of(s0, s1, s2, j + 4) & 63;
  } else {
    const int b4 = byte_of(s0, s1, s2, j + 4);
    sc = (b4 & 0xF) | ((byte_of(s0, s1, s2, j - 4) >> 6) << 4);
    m = (b4 >> 4) | ((byte_of(s0, s1, s2, j) >> 6) << 4);
  }
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
