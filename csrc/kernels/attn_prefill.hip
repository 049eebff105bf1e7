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

}  // namespace

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

extern "C" int nls_attn_prefill(const void* q, long ldq, const void* kc, const void* vc, const int* block_tables,
                                int bt_stride, const int* qblocks, int nqb, int Hq, int Hkv, int D, int block_size,
                                float scale, void* out, long ldo, void* stream) {
  return attn_prefill_impl<__bf16>(q, ldq, kc, vc, block_tables, bt_stride, qblocks, nqb, Hq, Hkv, D, block_size,
                                   scale, out, ldo, stream);
}

// the same over an fp8 (OCP e4m3) K/V cache
extern "C" int nls_attn_prefill8(const void* q, long ldq, const void* kc, const void* vc, const int* block_tables,
                                 int bt_stride, const int* qblocks, int nqb, int Hq, int Hkv, int D, int block_size,
                                 float scale, void* out, long ldo, void* stream) {
  return attn_prefill_impl<uint8_t>(q, ldq, kc, vc, block_tables, bt_stride, qblocks, nqb, Hq, Hkv, D, block_size,
                                    scale, out, ldo, stream);
}
