// Causal flash attention for prefill over the paged KV cache, on MFMA (gfx950).
// SURVEY.md §2F attn_prefill.
//
// Work item = one "query block": up to 16 * NSUB consecutive prompt tokens of ONE sequence
// (t0, ntok, seq, pos0) -- the engine cuts each sequence's prefill chunk into such blocks
// (ops.prefill_blocks, PREFILL_QT). Workgroup = (query block, kv head, quad of query heads): its 4
// waves are 4 query heads of the same GQA group and each wave runs the block's NSUB 16-token
// sub-tiles, so every K/V tile staged in LDS serves 4 heads x 16 * NSUB tokens (NSUB = 2: half the
// K/V staging per query of 16-token blocks).
//
// Per 96-key tile (KT) and wave sub-tile (16 tokens x 1 head):
//   S^T = K Q^T    v_mfma_f32_16x16x32_bf16, A = K rows from LDS, B = Q^T from registers.
//                  The transposed product puts one TOKEN per lane column, so each lane holds
//                  4 consecutive keys of its token per 16-key n-tile: the row max / sum of the
//                  online softmax need only 2 cross-lane shuffles.
//   O += P V       A = P straight from the S^T accumulators (no LDS round trip): lane (g, r)
//                  holds token r's keys {4g..4g+3, 16+4g..16+4g+3} of a 32-key group, and the
//                  MFMA's K order is free, so B = V rows in that same key order, read from a
//                  TRANSPOSED V tile in LDS (Vt[d][key], two 8-byte reads per fragment).
// Softmax in base 2 with the scale folded in; rows past ntok are computed but never stored.
#include "common.h"

namespace {

constexpr float LOG2E_P = 1.4426950408889634f;

constexpr int NSUB = 2;            // 16-token sub-tiles per query block (ops.PREFILL_QT = 16 * NSUB)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

template <int D, typename KV>
__global__ __launch_bounds__(256, 2) void attn_prefill_kernel(const __bf16* __restrict__ q, long ldq,
                                                           const KV* __restrict__ kc,
                                                           const KV* __restrict__ vc,
                                                           const int* __restrict__ block_tables, int bt_stride,
                                                           const int* __restrict__ qblocks, int Hkv, int G, int bs,
                                                           float scale, act_t* __restrict__ out, long ldo) {
  constexpr int KT = 96;           // keys per tile (a multiple of 32)
  constexpr int NT16 = KT / 16;    // 16-key n-tiles of S^T per tile
  constexpr int KSTR = D + 8;      // K tile row stride (elements): conflict-free ds_read_b128
  constexpr int VSTR = KT + 8;     // Vt row stride (keys): conflict-free ds_read_b64
  constexpr int NKK = D / 32;      // k-steps of S^T over the head dim
  constexpr int NDT = D / 16;      // n-tiles of O over the head dim
  __shared__ __attribute__((aligned(16))) __bf16 Ks[KT * KSTR];
  __shared__ __attribute__((aligned(16))) __bf16 Vt[D * VSTR];

  const int qb = blockIdx.x, hk = blockIdx.y, hq = blockIdx.z;
  const int t0 = qblocks[qb * 4], ntok = qblocks[qb * 4 + 1], seq = qblocks[qb * 4 + 2],
            pos0 = qblocks[qb * 4 + 3];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int head = hk * G + hq * 4 + wave;
  const int* bt = block_tables + (size_t)seq * bt_stride;
  const float sl2 = scale * LOG2E_P;

  // per sub-tile u: tokens 16u .. 16u + 15 of the block (lane column r = token 16u + r)
  bf16x8 qf[NSUB][NKK];
  float m[NSUB], l[NSUB];
  f32x4 o[NSUB][NDT];
#pragma unroll
  for (int u = 0; u < NSUB; ++u) {
    const __bf16* qrow = q + (size_t)(t0 + min(16 * u + r, ntok - 1)) * ldq + (size_t)head * D;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) qf[u][kk] = *reinterpret_cast<const bf16x8*>(qrow + kk * 32 + 8 * g);
    m[u] = -INFINITY;
    l[u] = 0.f;
#pragma unroll
    for (int i = 0; i < NDT; ++i) o[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int nkeys = pos0 + ntok;
  for (int k0 = 0; k0 < nkeys; k0 += KT) {
    __syncthreads();                           // previous tile fully consumed
    // ---- stage K [64][D] and V^T [D][64] of keys k0..k0+63 (zero past the end)
    for (int c = threadIdx.x; c < KT * (D / 8); c += 256) {
      const int key = c / (D / 8), ch = c % (D / 8);
      const int p = k0 + key;
      u32x4 v = u32x4{0u, 0u, 0u, 0u};
      if (p < nkeys) {
        const long slot = (long)bt[p / bs] * bs + p % bs;
        v = KVRaw<KV>::bf16(KVRaw<KV>::ld(kc + ((size_t)slot * Hkv + hk) * D + ch * 8));
      }
      *reinterpret_cast<u32x4*>(Ks + key * KSTR + ch * 8) = v;
    }
    for (int c = threadIdx.x; c < (KT / 2) * (D / 8); c += 256) {
      const int kp = c / (D / 8), ch = c % (D / 8);
      const int p = k0 + 2 * kp;
      u32x4 va = u32x4{0u, 0u, 0u, 0u}, vb = u32x4{0u, 0u, 0u, 0u};
      if (p < nkeys) {
        const long slot = (long)bt[p / bs] * bs + p % bs;
        va = KVRaw<KV>::bf16(KVRaw<KV>::ld(vc + ((size_t)slot * Hkv + hk) * D + ch * 8));
      }
      if (p + 1 < nkeys) {
        const long slot = (long)bt[(p + 1) / bs] * bs + (p + 1) % bs;
        vb = KVRaw<KV>::bf16(KVRaw<KV>::ld(vc + ((size_t)slot * Hkv + hk) * D + ch * 8));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // dims ch*8+2j and ch*8+2j+1: pair the two keys per dim into one 4-byte store
        const uint32_t lo = (va[j] & 0xFFFFu) | (vb[j] << 16);
        const uint32_t hi = (va[j] >> 16) | (vb[j] & 0xFFFF0000u);
        *reinterpret_cast<uint32_t*>(Vt + (ch * 8 + 2 * j) * VSTR + 2 * kp) = lo;
        *reinterpret_cast<uint32_t*>(Vt + (ch * 8 + 2 * j + 1) * VSTR + 2 * kp) = hi;
      }
    }
    __syncthreads();

#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
      if (16 * u >= ntok || k0 > pos0 + 16 * u + 15) continue;     // no token / every key of the tile is masked
      const int qpos = pos0 + 16 * u + r;       // this lane's token (column of S^T)
      const bool qvalid = 16 * u + r < ntok;
      // ---- S^T = K Q^T : s[nt][i] = S[token r][key k0 + nt*16 + 4g + i]
      f32x4 s[NT16];
#pragma unroll
      for (int nt = 0; nt < NT16; ++nt) {
        s[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(Ks + (nt * 16 + r) * KSTR + kk * 32 + 8 * g);
          s[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[u][kk], s[nt], 0, 0, 0);
        }
      }
      // ---- causal mask + online softmax (base 2)
      float mx = -INFINITY;
#pragma unroll
      for (int nt = 0; nt < NT16; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = k0 + nt * 16 + 4 * g + i;
          const float v = (qvalid && key <= qpos) ? s[nt][i] * sl2 : -INFINITY;
          s[nt][i] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m[u], mx);
      const float alpha = (mn == -INFINITY) ? 1.f : exp2f(m[u] - mn);
      float ps = 0.f;
#pragma unroll
      for (int nt = 0; nt < NT16; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = (mn == -INFINITY) ? 0.f : exp2f(s[nt][i] - mn);
          s[nt][i] = p;
          ps += p;
        }
      l[u] = l[u] * alpha + ps;
      m[u] = mn;
      // O rows are tokens 4g+i: their alpha lives in lane column 4g+i
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float ai = __shfl(alpha, 4 * g + i, 64);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) o[u][dt][i] *= ai;
      }
      // ---- O += P V over the tile's 32-key groups
#pragma unroll
      for (int kg = 0; kg < KT / 32; ++kg) {
        bf16x8 pa;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pa[i] = (__bf16)s[2 * kg][i];
          pa[4 + i] = (__bf16)s[2 * kg + 1][i];
        }
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const __bf16* vrow = Vt + (dt * 16 + r) * VSTR + kg * 32 + 4 * g;
          const uint2 lo = *reinterpret_cast<const uint2*>(vrow);
          const uint2 hi = *reinterpret_cast<const uint2*>(vrow + 16);
          u32x4 bw = u32x4{lo.x, lo.y, hi.x, hi.y};
          const bf16x8 b = __builtin_bit_cast(bf16x8, bw);
          o[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, b, o[u][dt], 0, 0, 0);
        }
      }
    }
  }
  // ---- normalise and store: lane holds O[token 16u + 4g+i][dt*16 + r]
#pragma unroll
  for (int u = 0; u < NSUB; ++u) {
    float lu = l[u];
    lu += __shfl_xor(lu, 16, 64);
    lu += __shfl_xor(lu, 32, 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int tok = 16 * u + 4 * g + i;
      const float li = __shfl(lu, 4 * g + i, 64);
      if (tok < ntok) {
        const float inv = li > 0.f ? 1.f / li : 0.f;
        act_t* orow = out + (size_t)(t0 + tok) * ldo + (size_t)head * D;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) orow[dt * 16 + r] = (act_t)(o[u][dt][i] * inv);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------------------
// attn_prefill2: the 8-wave, 32x32x16 structure (cdna_hip_programming.md "Fused attention prefill": swapped
// QK^T so a lane owns one query row, in-register softmax, V^T read by ds_read_b64_tr_b16, register-staged
// K/V split into issue-early / write-late, one barrier per tile).
//
// Workgroup = (kv head, quad of query heads, 64-token query block): wave w = head (w & 3) x tokens
// 32 (w >> 2) .. +31, so every 64-key K/V tile staged in LDS serves 4 heads x 64 tokens = 256 query rows
// (twice attn_prefill's 128). Per tile and wave:
//   S^T = K Q^T   2 key blocks x D/16 v_mfma_f32_32x32x16_bf16; lane l: token l & 31, keys (r & 3) +
//                 8 (r >> 2) + 4 (l >> 5) of each 32-key block -> 32 scores per lane, the row's other 32
//                 in lane l ^ 32 (one shuffle per max).
//   O^T += V^T P^T  4 k-steps x D/32 MFMAs with A = V^T (two transposed LDS reads per fragment, rows in
//                 the key order the accumulators already have) and B = P^T straight from the S^T
//                 registers -- so O's token is the lane's own and its rescale is lane-local.
// K rows are XOR-swizzled per 16-byte chunk (row & 15: conflict-free ds_read_b128 down 16 rows), V rows
// by 4 (key & 3) (conflict-free transposed reads of 4 keys x 32 dims per half wave). The next tile's K/V
// are loaded into registers while this tile computes (paged: one block-table lookup per key) and written
// to the other LDS buffer after it; the rescale of O is skipped when no row max grew.
// Grid: one workgroup per CU (64 KiB LDS, 2 waves per SIMD); blockIdx -> kv head first, so every query
// block of a kv head runs on one XCD and shares its K/V through that XCD's L2.
template <int D, typename KV>
__global__ __launch_bounds__(512, 1) void attn_prefill2_kernel(const __bf16* __restrict__ q, long ldq,
                                                            const KV* __restrict__ kc, const KV* __restrict__ vc,
                                                            const int* __restrict__ block_tables, int bt_stride,
                                                            const int* __restrict__ qblocks, int nqb, int Hkv, int G,
                                                            int bs_shift, float scale, act_t* __restrict__ out,
                                                            long ldo) {
  constexpr int KT = 64;                 // keys per tile
  constexpr int NCH = D / 8;             // 16-byte chunks per K / V row
  constexpr int ROWB = D * 2;            // bytes per LDS row
  constexpr int TILEB = KT * ROWB;       // one K (or V) tile
  constexpr int NKS = D / 16;            // k-steps of S^T over the head dim
  constexpr int NDB = D / 32;            // 32-dim blocks of O^T
  constexpr int NLD = KT * NCH / 512;    // staging chunks per thread per K (and per V) tile
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * 2 * TILEB];   // [buf][K | V]

  const int nq4 = G / 4;
  const int bi = blockIdx.x;
  const int hk = bi % Hkv;
  const int rest = bi / Hkv;
  const int hq4 = rest % nq4;
  const int qb = nqb - 1 - rest / nq4;   // heaviest (latest) query blocks first
  const int t0 = qblocks[qb * 4], ntok = qblocks[qb * 4 + 1], seq = qblocks[qb * 4 + 2], pos0 = qblocks[qb * 4 + 3];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, tl = lane & 31;
  const int head = hk * G + hq4 * 4 + (wave & 3);
  const int tw0 = 32 * (wave >> 2);      // the wave's first token of the block
  const int* bt = block_tables + (size_t)seq * bt_stride;
  const int bsm = (1 << bs_shift) - 1;
  const float sl2 = scale * LOG2E_P;
  const int nkeys = pos0 + ntok;
  const int ntile = (nkeys + KT - 1) / KT;
  const int wlast = pos0 + min(tw0 + 31, ntok - 1);   // the wave's last valid token position
  const bool wact = tw0 < ntok;

  // ---- Q^T fragments: token tw0 + tl, dims 16 ks + 8 h .. +7
  bf16x8 qf[NKS];
  {
    const __bf16* qrow = q + (size_t)(t0 + min(tw0 + tl, ntok - 1)) * ldq + (size_t)head * D;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qrow + 16 * ks + 8 * h);
  }
  const int qpos = pos0 + tw0 + tl;

  // ---- staging: thread tid moves chunks e = tid + 512 i (key e / NCH, chunk e % NCH) of K and of V
  typename KVRaw<KV>::raw kr[NLD], vr[NLD];
  auto load_tile = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int e = tid + 512 * i, key = e / NCH, ch = e % NCH;
      const int p = t * KT + key;
      if (p < nkeys) {
        const size_t off = ((size_t)(bt[p >> bs_shift] << bs_shift | (p & bsm)) * Hkv + hk) * D + ch * 8;
        kr[i] = KVRaw<KV>::ld(kc + off);
        vr[i] = KVRaw<KV>::ld(vc + off);
      } else {
        kr[i] = typename KVRaw<KV>::raw{};
        vr[i] = typename KVRaw<KV>::raw{};
      }
    }
  };
  auto store_tile = [&](int buf) __attribute__((always_inline)) {
    uint8_t* kb = lds + buf * 2 * TILEB;
    uint8_t* vb = kb + TILEB;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int e = tid + 512 * i, key = e / NCH, ch = e % NCH;
      *reinterpret_cast<u32x4*>(kb + key * ROWB + ((ch ^ (key & (NCH - 1) & 15)) << 4)) = KVRaw<KV>::bf16(kr[i]);
      *reinterpret_cast<u32x4*>(vb + key * ROWB + ((ch ^ (((key & 3) << 2) & (NCH - 1))) << 4)) = KVRaw<KV>::bf16(vr[i]);
    }
  };

  f32x16 o[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) o[i] = f32x16{};
  float m = -INFINITY, l = 0.f;

  load_tile(0);
  store_tile(0);
  __syncthreads();
  // V^T fragment read: lane (group of 16: q = (l & 15) >> 2 row, p = l & 3 column quad) supplies row
  // kbase + q (and + 8), dims 32 db + 16 ((l >> 4) & 1) + 4 p
  const int vq = (lane & 15) >> 2, vp = lane & 3, vhalf = (lane >> 4) & 1;
  for (int t = 0; t < ntile; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntile) load_tile(t + 1);      // issue early: lands while this tile computes
    const int k0 = t * KT;
    if (wact && k0 <= wlast) {
      const uint8_t* kb = lds + cur * 2 * TILEB;
      const uint8_t* vb = kb + TILEB;
      // ---- S^T = K Q^T
      f32x16 s[2];
#pragma unroll
      for (int kb2 = 0; kb2 < 2; ++kb2) {
        s[kb2] = f32x16{};
        const int key = 32 * kb2 + tl;
        const uint8_t* krow = kb + key * ROWB;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const int ch = 2 * ks + h;
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(krow + ((ch ^ (key & (NCH - 1) & 15)) << 4));
          s[kb2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[ks], s[kb2], 0, 0, 0);
        }
      }
      // ---- causal mask (only tiles that reach past the wave's first token) + row max
      float mx = -INFINITY;
      if (k0 + KT - 1 > pos0 + tw0) {
#pragma unroll
        for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + 32 * kb2 + (r & 3) + 8 * (r >> 2) + 4 * h;
            const float v = key <= qpos ? s[kb2][r] : -INFINITY;
            s[kb2][r] = v;
            mx = fmaxf(mx, v);
          }
      } else {
#pragma unroll
        for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kb2][r]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx);
      if (!__all(mn == m)) {                 // some row's max grew: rescale (rare after the first tiles)
        const float alpha = (mn == -INFINITY) ? 1.f : __builtin_amdgcn_exp2f((m - mn) * sl2);
        l *= alpha;
#pragma unroll
        for (int db = 0; db < NDB; ++db) o[db] *= alpha;
        m = mn;
      }
      const float nb = (m == -INFINITY) ? 0.f : -m * sl2;
      // ---- P = exp2((s - m) * scale log2e), row partial sums, and O^T += V^T P^T per 16-key step
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int kb2 = ks >> 1, r0 = 8 * (ks & 1);
        bf16x8 pb;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[kb2][r0 + j], sl2, nb));
          l += p;
          pb[j] = (__bf16)p;
        }
        // keys of this step in the fragment's k order: 32 kb2 + 16 (ks & 1) + 4 h + {0..3, 8..11}
        const int kbase = 32 * kb2 + 16 * (ks & 1) + 4 * h;
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
          const int ch = 4 * db + 2 * vhalf + (vp >> 1);
          const int k1 = kbase + vq, k2 = kbase + 8 + vq;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(vb + k1 * ROWB + ((ch ^ (((k1 & 3) << 2) & (NCH - 1))) << 4) + 8 * (vp & 1)));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(vb + k2 * ROWB + ((ch ^ (((k2 & 3) << 2) & (NCH - 1))) << 4) + 8 * (vp & 1)));
          const s16x8 a8 = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a8), pb, o[db], 0, 0, 0);
        }
      }
    }
    if (t + 1 < ntile) {
      store_tile(cur ^ 1);                    // write late: the other buffer was last read in tile t - 1
    }
    __syncthreads();
  }
  // ---- normalise and store: lane holds O[token tw0 + tl][32 db + 8 g + 4 h + 0..3] in o[db][4 g .. 4 g + 3]
  l += __shfl_xor(l, 32, 64);
  const int tok = tw0 + tl;
  if (wact && tok < ntok) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    act_t* orow = out + (size_t)(t0 + tok) * ldo + (size_t)head * D;
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<h4*>(orow + 32 * db + 8 * g + 4 * h) =
            h4{(act_t)(o[db][4 * g] * inv), (act_t)(o[db][4 * g + 1] * inv), (act_t)(o[db][4 * g + 2] * inv),
               (act_t)(o[db][4 * g + 3] * inv)};
  }
}

}  // namespace

template <typename KV>
int attn_prefill2_impl(const void* q, long ldq, const void* kc, const void* vc, const int* block_tables, int bt_stride,
                       const int* qblocks, int nqb, int Hq, int Hkv, int D, int block_size, float scale, void* out,
                       long ldo, void* stream) {
  if (Hq % Hkv || (Hq / Hkv) % 4 || (D != 64 && D != 128) || nqb < 1 || block_size < 1 ||
      (block_size & (block_size - 1)))
    return -1;
  const int G = Hq / Hkv;
  const int bs_shift = __builtin_ctz(block_size);
  dim3 grid(nqb * Hkv * (G / 4));
  hipStream_t st = (hipStream_t)stream;
  if (D == 128)
    hipLaunchKernelGGL((attn_prefill2_kernel<128, KV>), grid, dim3(512), 0, st, (const __bf16*)q, ldq, (const KV*)kc,
                       (const KV*)vc, block_tables, bt_stride, qblocks, nqb, Hkv, G, bs_shift, scale, (act_t*)out, ldo);
  else
    hipLaunchKernelGGL((attn_prefill2_kernel<64, KV>), grid, dim3(512), 0, st, (const __bf16*)q, ldq, (const KV*)kc,
                       (const KV*)vc, block_tables, bt_stride, qblocks, nqb, Hkv, G, bs_shift, scale, (act_t*)out, ldo);
  return (int)hipGetLastError();
}

extern "C" int nls_attn_prefill(const void* q, long ldq, const void* kc, const void* vc, const int* block_tables,
                                 int bt_stride, const int* qblocks, int nqb, int Hq, int Hkv, int D, int block_size,
                                 float scale, void* out, long ldo, void* stream) {
  return attn_prefill2_impl<__bf16>(q, ldq, kc, vc, block_tables, bt_stride, qblocks, nqb, Hq, Hkv, D, block_size,
                                    scale, out, ldo, stream);
}

extern "C" int nls_attn_prefill8(const void* q, long ldq, const void* kc, const void* vc, const int* block_tables,
                                   int bt_stride, const int* qblocks, int nqb, int Hq, int Hkv, int D, int block_size,
                                   float scale, void* out, long ldo, void* stream) {
  return attn_prefill2_impl<uint8_t>(q, ldq, kc, vc, block_tables, bt_stride, qblocks, nqb, Hq, Hkv, D, block_size,
                                     scale, out, ldo, stream);
}

template <typename KV>
int attn_prefill_impl(const void* q, long ldq, const void* kc, const void* vc, const int* block_tables, int bt_stride,
                      const int* qblocks, int nqb, int Hq, int Hkv, int D, int block_size, float scale, void* out,
                      long ldo, void* stream) {
  if (Hq % Hkv || (Hq / Hkv) % 4 || (D != 64 && D != 128) || nqb < 1) return -1;
  const int G = Hq / Hkv;
  dim3 grid(nqb, Hkv, G / 4);
  hipStream_t st = (hipStream_t)stream;
  if (D == 128)
    hipLaunchKernelGGL((attn_prefill_kernel<128, KV>), grid, dim3(256), 0, st, (const __bf16*)q, ldq, (const KV*)kc,
                       (const KV*)vc, block_tables, bt_stride, qblocks, Hkv, G, block_size, scale, (act_t*)out, ldo);
  else
    hipLaunchKernelGGL((attn_prefill_kernel<64, KV>), grid, dim3(256), 0, st, (const __bf16*)q, ldq, (const KV*)kc,
                       (const KV*)vc, block_tables, bt_stride, qblocks, Hkv, G, block_size, scale, (act_t*)out, ldo);
  return (int)hipGetLastError();
}

// the first MFMA prefill kernel (4 waves, 16x16x32, 32-token query blocks): kept for A/B (NLS_PREFILL_V1=1)
extern "C" int nls_attn_prefill_v1(const void* q, long ldq, const void* kc, const void* vc, const int* block_tables,
                                   int bt_stride, const int* qblocks, int nqb, int Hq, int Hkv, int D, int block_size,
                                   float scale, void* out, long ldo, void* stream) {
  return attn_prefill_impl<__bf16>(q, ldq, kc, vc, block_tables, bt_stride, qblocks, nqb, Hq, Hkv, D, block_size,
                                   scale, out, ldo, stream);
}

// the same over an fp8 (OCP e4m3) K/V cache
extern "C" int nls_attn_prefill_v18(const void* q, long ldq, const void* kc, const void* vc, const int* block_tables,
                                    int bt_stride, const int* qblocks, int nqb, int Hq, int Hkv, int D, int block_size,
                                    float scale, void* out, long ldo, void* stream) {
  return attn_prefill_impl<uint8_t>(q, ldq, kc, vc, block_tables, bt_stride, qblocks, nqb, Hq, Hkv, D, block_size,
                                    scale, out, ldo, stream);
}
